// hbm_ceiling.hip — calibration: the fastest in-place read-modify-write stream
// this MI355X sustains, to price the rank-1 update against a measured ceiling
// as well as the 8 TB/s spec.  Same traffic shape as the update (every fp64
// element read once and written once, 16 B per lane per access), no pivot
// logic.  Build: make tools;  run: build/hbm_ceiling [GiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));         \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

// grid-stride: each lane updates 16 B per step, U steps in flight
template <bool NT, int U>
__global__ __launch_bounds__(256) void rmw_gridstride(double* __restrict__ p, size_t n2, double f) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n2; i += U * stride) {
        d2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = NT ? __builtin_nontemporal_load((const d2*)p + i + u * stride)
                      : ((const d2*)p)[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u].x = __builtin_fma(-f, 1.0, v[u].x);
            v[u].y = __builtin_fma(-f, 1.0, v[u].y);
            if (NT)
                __builtin_nontemporal_store(v[u], (d2*)p + i + u * stride);
            else
                ((d2*)p)[i + u * stride] = v[u];
        }
    }
    for (; i < n2; i += stride) ((d2*)p)[i] = ((const d2*)p)[i];
}

// block-contiguous chunks: workgroup b owns a contiguous 4 KiB x R span
template <bool NT>
__global__ __launch_bounds__(256) void rmw_chunks(double* __restrict__ p, size_t n2, int rows,
                                                  double f) {
    const size_t base = (size_t)blockIdx.x * 256 * rows;
    for (int r = 0; r < rows; ++r) {
        const size_t i = base + (size_t)r * 256 + threadIdx.x;
        if (i >= n2) return;
        d2 v = NT ? __builtin_nontemporal_load((const d2*)p + i) : ((const d2*)p)[i];
        v.x = __builtin_fma(-f, 1.0, v.x);
        v.y = __builtin_fma(-f, 1.0, v.y);
        if (NT)
            __builtin_nontemporal_store(v, (d2*)p + i);
        else
            ((d2*)p)[i] = v;
    }
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? std::atof(argv[1]) : 16.0;
    const size_t bytes = (size_t)(gib * (1ull << 30)) / 4096 * 4096;
    const size_t n2 = bytes / 16;
    double* p = nullptr;
    CK(hipMalloc(&p, bytes));
    CK(hipMemset(p, 0, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char* name, auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int k = 0; k < 5; ++k) {
            CK(hipEventRecord(a));
            launch();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
        }
        std::printf("{\"kernel\": \"%s\", \"bytes_rw\": %zu, \"best_ms\": %.4f, \"GBps\": %.1f}\n", name,
                    2 * bytes, best, 2.0 * bytes / (best * 1e-3) / 1e9);
    };
    for (int blocks : {2048, 4096, 8192}) {
        char nm[96];
        std::snprintf(nm, sizeof nm, "gridstride nt U4 blocks=%d", blocks);
        run(nm, [&] { rmw_gridstride<true, 4><<<blocks, 256>>>(p, n2, 0.0); });
        std::snprintf(nm, sizeof nm, "gridstride plain U4 blocks=%d", blocks);
        run(nm, [&] { rmw_gridstride<false, 4><<<blocks, 256>>>(p, n2, 0.0); });
        std::snprintf(nm, sizeof nm, "gridstride nt U1 blocks=%d", blocks);
        run(nm, [&] { rmw_gridstride<true, 1><<<blocks, 256>>>(p, n2, 0.0); });
    }
    for (int rows : {4, 8, 32}) {
        char nm[96];
        const size_t nb = (n2 + 256 * (size_t)rows - 1) / (256 * (size_t)rows);
        std::snprintf(nm, sizeof nm, "chunks nt rows=%d", rows);
        run(nm, [&] { rmw_chunks<true><<<(unsigned)nb, 256>>>(p, n2, rows, 0.0); });
        std::snprintf(nm, sizeof nm, "chunks plain rows=%d", rows);
        run(nm, [&] { rmw_chunks<false><<<(unsigned)nb, 256>>>(p, n2, rows, 0.0); });
    }
    CK(hipFree(p));
    return 0;
}
