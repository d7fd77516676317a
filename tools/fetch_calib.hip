// fetch_calib.hip — calibration of the FETCH_SIZE counter ("calibrate FETCH_SIZE for
// buffer_load_b64 against a known-byte stream before quoting the traffic ratio").  Each kernel reads
// a known number of bytes exactly once, with one of the three access types the tableau passes use:
//   b64   8 B per lane (buffer_load_b64: form 21's tableau loads)
//   b128  16 B per lane (global_load_dwordx4: the eager update, forms 4 / 20)
//   glds  16 B per lane straight into LDS (global_load_lds_dwordx4: form 23's ring, the chain rings)
// and writes 8 B per workgroup.  rocprofv3 --pmc FETCH_SIZE (one counter pass per run) then gives
// FETCH_SIZE x 1024 / bytes for each, the factor tools/pmc_summary.py must apply.
//   build: hipcc --offload-arch=gfx950 -O3 -o build/fetch_calib tools/fetch_calib.hip
//   run:   build/fetch_calib <b64|b128|glds> [GiB]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef double d2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

// one contiguous 1 KiB chunk per wave per step (64 lanes x 16 B, or 2 steps of 64 x 8 B), grid-stride
__global__ __launch_bounds__(256) void rd_b64(const double* __restrict__ p, size_t n, double* out) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    double acc = 0.0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        acc += __builtin_nontemporal_load(p + i);
    if (acc == 1.25) out[blockIdx.x] = acc;   // (never: the data are zeros)
}

__global__ __launch_bounds__(256) void rd_b128(const d2* __restrict__ p, size_t n2, double* out) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    double acc = 0.0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += stride) {
        const d2 v = __builtin_nontemporal_load(p + i);
        acc += v.x + v.y;
    }
    if (acc == 1.25) out[blockIdx.x] = acc;
}

__device__ __forceinline__ void glds16(const void* g, uint32_t m0) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}

// each wave streams 1 KiB chunks into its own LDS slot (4 in flight), then reads one double back
__global__ __launch_bounds__(256) void rd_glds(const d2* __restrict__ p, size_t n2, double* out) {
    __shared__ double ring[4][4][128];   // [wave][slot][1 KiB]
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const size_t nw = (size_t)gridDim.x * 4, wid = (size_t)blockIdx.x * 4 + w;
    const size_t nchunks = n2 / 64;
    double acc = 0.0;
    int s = 0;
    for (size_t c = wid; c < nchunks; c += nw) {
        const uint32_t m0 = __builtin_amdgcn_readfirstlane(
            (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)&ring[w][s][0]);
        glds16(p + c * 64 + lane, m0);
        s = (s + 1) & 3;
        if (s == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            acc += ring[w][3][lane];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (acc == 1.25) out[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
    const char* kind = argc > 1 ? argv[1] : "b64";
    const double gib = argc > 2 ? std::atof(argv[2]) : 4.0;
    const size_t bytes = (size_t)(gib * (double)(1ull << 30)) / 4096 * 4096;
    void* p = nullptr;
    double* out = nullptr;
    CK(hipMalloc(&p, bytes));
    CK(hipMemset(p, 0, bytes));
    const int blocks = 256 * 8;
    CK(hipMalloc(&out, sizeof(double) * blocks));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipEventRecord(e0));
        if (!std::strcmp(kind, "b64"))
            rd_b64<<<blocks, 256>>>((const double*)p, bytes / 8, out);
        else if (!std::strcmp(kind, "b128"))
            rd_b128<<<blocks, 256>>>((const d2*)p, bytes / 16, out);
        else
            rd_glds<<<blocks, 256>>>((const d2*)p, bytes / 16, out);
        CK(hipGetLastError());
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"kind\": \"%s\", \"bytes\": %zu, \"ms\": %.4f, \"gbs\": %.1f}\n", kind, bytes, ms,
                    bytes / (ms * 1e-3) / 1e9);
    }
    CK(hipFree(p));
    CK(hipFree(out));
    return 0;
}
