// mall_probe.hip — does a streaming kernel's cache policy decide whether a small table stays in the
// 256 MiB Infinity Cache (MALL)?  The lookahead chain re-reads ~50 MB per pivot (the sealed block's
// coefficients and pivot rows) while the rank-64 pass streams the whole tableau beside it; if the
// pass's loads and stores could stream without allocating in the MALL, the chain's re-reads would hit.
//
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/mall_probe tools/mall_probe.hip
//   run:   tools/bin/mall_probe [table_MB] [stream_MB]
//
// For each policy (buffer-op aux bits of the stream's loads and stores: 0 default, 1 sc0, 2 nt,
// 16 sc1, 17 sc0 sc1, 18 nt sc1, 3 sc0 nt, 19 sc0 nt sc1): read the table (warm), stream-copy
// stream_MB through that policy, then time one read of the table.  A table still in the MALL reads
// at the "no stream" rate; an evicted one at the HBM rate.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>


#define CK(x)                                                                             \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

__device__ inline __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, 0x00020000);
}

// table read: every lane sums its 16-B elements (grid-stride), one store per lane at the end
__global__ __launch_bounds__(256) void read_kernel(const d2* __restrict__ a, size_t n, double* out) {
    d2 s = {0.0, 0.0};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
    out[(size_t)blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

// stream copy src -> dst with the given aux bits on both the loads and the stores; 1 GiB windows
// through buffer resources (each window < 4 GiB), grid-stride within a window
template <int AUX>
__global__ __launch_bounds__(256) void stream_kernel(const double* __restrict__ src, double* __restrict__ dst,
                                                     size_t bytes) {
    const size_t win = (size_t)1 << 30;
    for (size_t w0 = 0; w0 < bytes; w0 += win) {
        const uint32_t wb = (uint32_t)std::min(win, bytes - w0);
        const __amdgpu_buffer_rsrc_t rs = rsrc((const char*)src + w0, wb);
        const __amdgpu_buffer_rsrc_t rd = rsrc((char*)dst + w0, wb);
        for (uint32_t off = (blockIdx.x * 256u + threadIdx.x) * 16u; off < wb; off += gridDim.x * 256u * 16u) {
            const d2 v = __builtin_bit_cast(d2, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, AUX));
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                                   rd, off, 0, AUX);
        }
    }
}

// latency: one wave, lane 0 follows a chain of dependent loads: a random cycle over every 128-B line
// of the table, continued from where the previous launch stopped (state[1]), so each launch meets
// lines last touched a whole table ago: out of the 4 MiB L2, in the Infinity Cache
__global__ __launch_bounds__(64) void chase_kernel(const uint64_t* __restrict__ next, int hops, uint64_t* state,
                                                   long long* cycles) {
    if (threadIdx.x != 0) return;
    uint64_t i = state[1];
    const long long t0 = wall_clock64();
    for (int h = 0; h < hops; ++h) i = __builtin_nontemporal_load(next + i);
    cycles[0] = wall_clock64() - t0;
    state[1] = i;
}

typedef void (*StreamFn)(const double*, double*, size_t);

template <int AUX>
void launch_stream(const double* s, double* d, size_t bytes) {
    stream_kernel<AUX><<<256 * 8, 256>>>(s, d, bytes);
}

int main(int argc, char** argv) {
    const size_t table_mb = argc > 1 ? std::atoll(argv[1]) : 48;
    const size_t stream_mb = argc > 2 ? std::atoll(argv[2]) : 2048;
    const size_t tb = table_mb << 20, sb = stream_mb << 20;
    double *table, *src, *dst, *out;
    CK(hipMalloc(&table, tb));
    CK(hipMalloc(&src, sb));
    CK(hipMalloc(&dst, sb));
    CK(hipMalloc(&out, sizeof(double) * 256 * 1024));
    CK(hipMemset(table, 0, tb));
    CK(hipMemset(src, 0, sb));
    CK(hipMemset(dst, 0, sb));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t n2 = tb / 16;
    auto read_ms = [&]() {
        CK(hipEventRecord(e0, 0));
        read_kernel<<<1024, 256>>>((const d2*)table, n2, out);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms;
    };
    struct P { int aux; const char* name; StreamFn fn; };
    const P pols[] = {{-1, "no stream", nullptr},
                      {0, "default", launch_stream<0>},
                      {1, "sc0", launch_stream<1>},
                      {2, "nt", launch_stream<2>},
                      {3, "sc0 nt", launch_stream<3>},
                      {16, "sc1", launch_stream<16>},
                      {17, "sc0 sc1", launch_stream<17>},
                      {18, "nt sc1", launch_stream<18>},
                      {19, "sc0 nt sc1", launch_stream<19>}};
    if (argc > 4) {   // latency: dependent loads beside an nt stream of argv[3] workgroups
        const int nwg = std::atoi(argv[3]);
        const size_t nq = tb / 8, nl = tb / 128;
        std::vector<uint64_t> h(nq, 0), perm(nl);
        for (size_t k = 0; k < nl; ++k) perm[k] = k;
        uint64_t x = 12345;
        for (size_t k = nl - 1; k > 0; --k) {   // Fisher-Yates with a splitmix step
            x += 0x9e3779b97f4a7c15ull;
            uint64_t z = x;
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
            z ^= z >> 31;
            std::swap(perm[k], perm[z % (k + 1)]);
        }
        for (size_t k = 0; k < nl; ++k) h[perm[k] * 16] = perm[(k + 1) % nl] * 16;
        CK(hipMemcpy(table, h.data(), tb, hipMemcpyHostToDevice));
        CK(hipMemset(out, 0, 64));
        long long* cyc;
        CK(hipMalloc(&cyc, 64));
        int lo = 0, hi = 0;
        CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        hipStream_t sa, sbq;
        CK(hipStreamCreateWithPriority(&sa, hipStreamNonBlocking, lo));
        CK(hipStreamCreateWithPriority(&sbq, hipStreamNonBlocking, hi));
        const int hops = 2000;
        for (int rep = 0; rep < 4; ++rep) {
            for (int w = 0; w < 300; ++w)   // warm: the whole cycle, twice
                chase_kernel<<<1, 64, 0, sbq>>>((const uint64_t*)table, hops, (uint64_t*)out, cyc);
            CK(hipDeviceSynchronize());
            for (int r = 0; nwg > 0 && r < 12; ++r)   // ~40 ms of stream: every chase below runs beside it
                stream_kernel<2><<<nwg, 256, 0, sa>>>(src, dst, sb);
            std::vector<double> ns;
            for (int k = 0; k < 10; ++k) {
                chase_kernel<<<1, 64, 0, sbq>>>((const uint64_t*)table, hops, (uint64_t*)out, cyc);
                long long c = 0;
                CK(hipMemcpyAsync(&c, cyc, sizeof(c), hipMemcpyDeviceToHost, sbq));
                CK(hipStreamSynchronize(sbq));
                ns.push_back(c * 10.0 / hops);   // 100 MHz wall clock
            }
            CK(hipDeviceSynchronize());
            std::sort(ns.begin(), ns.end());
            std::printf("dependent-load latency beside an nt stream of %4d workgroups: median %.0f ns per hop (min %.0f)\n",
                        nwg, ns[5], ns[0]);
            std::fflush(stdout);
        }
        return 0;
    }
    if (argc > 3) {   // concurrent: table reads on a high-priority stream while an nt stream copies
        const int nwg = std::atoi(argv[3]);   // stream workgroups (throttle), 0 = no stream
        int lo = 0, hi = 0;
        CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
        hipStream_t sa, sbq;
        CK(hipStreamCreateWithPriority(&sa, hipStreamNonBlocking, lo));
        CK(hipStreamCreateWithPriority(&sbq, hipStreamNonBlocking, hi));
        std::vector<hipEvent_t> ev(41);
        for (auto& e : ev) CK(hipEventCreate(&e));
        for (int rep = 0; rep < 3; ++rep) {
            read_ms();
            hipEvent_t sa0, sa1;
            CK(hipEventCreate(&sa0));
            CK(hipEventCreate(&sa1));
            CK(hipEventRecord(sa0, sa));
            if (nwg > 0) stream_kernel<2><<<nwg, 256, 0, sa>>>(src, dst, sb);
            CK(hipEventRecord(sa1, sa));
            CK(hipEventRecord(ev[0], sbq));
            for (int k = 0; k < 40; ++k) {
                read_kernel<<<1024, 256, 0, sbq>>>((const d2*)table, n2, out);
                CK(hipEventRecord(ev[k + 1], sbq));
            }
            CK(hipDeviceSynchronize());
            std::vector<float> t(40);
            for (int k = 0; k < 40; ++k) CK(hipEventElapsedTime(&t[k], ev[k], ev[k + 1]));
            float sms = 0.0f;
            CK(hipEventElapsedTime(&sms, sa0, sa1));
            std::sort(t.begin(), t.end());
            std::printf("concurrent nt stream with %4d workgroups (%.3f ms, %5.0f GB/s): table reads median %.4f ms = %5.0f GB/s, min %.4f\n",
                        nwg, sms, nwg ? 2.0 * sb / sms / 1e6 : 0.0, t[20], tb / t[20] / 1e6, t[0]);
            std::fflush(stdout);
        }
        return 0;
    }
    std::printf("table %zu MB, stream %zu MB copied per trial\n", table_mb, stream_mb);
    for (int rep = 0; rep < 2; ++rep)
        for (const P& p : pols) {
            std::vector<float> t;
            float st_ms = 0.0f;
            for (int trial = 0; trial < 5; ++trial) {
                read_ms();
                read_ms();   // the table warm
                if (p.fn) {
                    CK(hipEventRecord(e0, 0));
                    p.fn(src, dst, sb);
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    CK(hipEventElapsedTime(&st_ms, e0, e1));
                }
                t.push_back(read_ms());
            }
            std::sort(t.begin(), t.end());
            std::printf("%-12s stream %7.3f ms (%5.0f GB/s)   table read after: median %.4f ms = %6.0f GB/s\n", p.name,
                        st_ms, p.fn ? 2.0 * sb / st_ms / 1e6 : 0.0, t[2], tb / t[2] / 1e6);
            std::fflush(stdout);
        }
    return 0;
}
