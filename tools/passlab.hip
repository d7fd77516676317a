// passlab.hip — standalone experiments on the deferred rank-K tableau pass
// (DESIGN.md §11), outside the session machinery: one tableau in HBM, one
// block of K dense steps (every row touched by every step), and variants of
// the per-element chain  t = fma(-C[i][l], P[l][j], t), l = 0..K-1.
//
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/bin/passlab tools/passlab.hip
//   run:   tools/bin/passlab [rows] [cols] [reps]      (defaults: C3, 32768 x 65537)
//
// Every variant is checked bit for bit against a one-thread-per-element
// reference kernel on a small tableau before the timed runs.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const double* cdptr;

__device__ inline double hrand(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    return (double)(x >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
}

__global__ void fill_kernel(double* a, int64_t n, uint64_t seed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        a[i] = hrand(seed * 0x100000001B3ull + (uint64_t)i);
}

// reference: one thread per element
__global__ void ref_kernel(const double* T, double* To, int64_t ld, int64_t rows, int64_t width, int K,
                           const double* Cr, const double* P) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = blockIdx.y;
    if (j >= width || i >= rows) return;
    double t = T[i * ld + j];
    for (int l = 0; l < K; ++l) t = __builtin_fma(-Cr[i * K + l], P[(int64_t)l * ld + j], t);
    To[i * ld + j] = t;
}

template <bool NT>
__device__ inline d2 ldv(const double* p) {
    if constexpr (NT) return __builtin_nontemporal_load((const d2*)p);
    else return *(const d2*)p;
}
template <bool NT>
__device__ inline void stv(double* p, d2 v) {
    if constexpr (NT) __builtin_nontemporal_store(v, (d2*)p);
    else *(d2*)p = v;
}

__device__ inline double rl(double v, int lane) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), lane);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// MODE 0: form 4 (coefficients by scalar loads, chunks of LC steps x U rows, double
//         buffered); 1: coefficients = kernel argument (no memory; wrong values, timing
//         only); 2: copy (no fma); 3: coefficients by ONE vector load per group (lane =
//         (row, step)) prefetched with the rows, moved to SGPRs with v_readlane.
// Workgroup = 256 lanes x V doubles of columns, band of rb rows; P[0..K)[V] in VGPRs.
template <bool NT, int K, int V, int U, int MODE>
__global__ __launch_bounds__(256) void f4_kernel(const double* __restrict__ T, double* __restrict__ To,
                                                 int64_t ld, int64_t rows, int64_t width,
                                                 const double* __restrict__ Cr, const double* __restrict__ P,
                                                 int rb, double cval) {
    const int64_t j = (int64_t)blockIdx.x * (256 * V) + threadIdx.x * V;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - V;
    double pr[K][V];
#pragma unroll
    for (int l = 0; l < K; ++l) {
        if constexpr (V == 2) {
            const d2 v = *(const d2*)(P + (int64_t)l * ld + jc);
            pr[l][0] = v.x;
            pr[l][1] = v.y;
        } else {
            pr[l][0] = P[(int64_t)l * ld + jc];
        }
    }
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    const int lane = threadIdx.x & 63;
    auto load = [&](double (&t)[U][V], int r0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double* p = T + (i0 + r0 + u) * ld + jc;
            if constexpr (V == 2) {
                const d2 v = ldv<NT>(p);
                t[u][0] = v.x;
                t[u][1] = v.y;
            } else {
                t[u][0] = NT ? __builtin_nontemporal_load(p) : *p;
            }
        }
    };
    auto store = [&](const double (&t)[U][V], int r0) {
        if (!colok) return;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            double* p = To + (i0 + r0 + u) * ld + j;
            if constexpr (V == 2) {
                d2 v;
                v.x = t[u][0];
                v.y = t[u][1];
                stv<NT>(p, v);
            } else {
                if (NT) __builtin_nontemporal_store(t[u][0], p);
                else *p = t[u][0];
            }
        }
    };
    constexpr int LC = (16 / U) < K ? (16 / U) : K;
    constexpr int NCV = (U * K + 63) / 64;   // MODE 3: coefficient doubles per lane per group
    auto chain_s = [&](double (&t)[U][V], const double (&f)[U][LC], int l0) {
#pragma unroll
        for (int l = 0; l < LC; ++l)
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int e = 0; e < V; ++e) t[u][e] = __builtin_fma(-f[u][l], pr[l0 + l][e], t[u][e]);
    };
    auto group = [&](double (&t)[U][V], int r0, const double (&cv)[NCV]) {
        if constexpr (MODE == 0) {
            const cdptr cb = (cdptr)(Cr + (i0 + r0) * K);
            double fa[U][LC], fb[U][LC];
            auto fetch = [&](double (&f)[U][LC], int l0) {
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int l = 0; l < LC; ++l) f[u][l] = cb[u * K + l0 + l];
            };
            fetch(fa, 0);
#pragma unroll
            for (int l0 = 0; l0 < K; l0 += 2 * LC) {
                __builtin_amdgcn_s_waitcnt(0xC07F);
                if (l0 + LC < K) fetch(fb, l0 + LC);
                __builtin_amdgcn_sched_barrier(0);
                chain_s(t, fa, l0);
                __builtin_amdgcn_sched_barrier(0);
                if (l0 + LC < K) {
                    __builtin_amdgcn_s_waitcnt(0xC07F);
                    if (l0 + 2 * LC < K) fetch(fa, l0 + 2 * LC);
                    __builtin_amdgcn_sched_barrier(0);
                    chain_s(t, fb, l0 + LC);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        } else if constexpr (MODE == 1) {
#pragma unroll
            for (int l = 0; l < K; ++l)
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int e = 0; e < V; ++e)
                        t[u][e] = __builtin_fma(-cval, pr[l][e], t[u][e]);
        } else if constexpr (MODE == 3) {
#pragma unroll
            for (int l = 0; l < K; ++l)
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int idx = u * K + l;
                    const double f = rl(cv[idx >> 6], idx & 63);
#pragma unroll
                    for (int e = 0; e < V; ++e) t[u][e] = __builtin_fma(-f, pr[l][e], t[u][e]);
                }
        }
        store(t, r0);
    };
    auto loadc = [&](double (&cv)[NCV], int r0) {
        if constexpr (MODE == 3) {
#pragma unroll
            for (int k = 0; k < NCV; ++k) {
                const int idx = k * 64 + lane;   // (u, l) = (idx / K, idx % K): row-major C is contiguous
                cv[k] = Cr[(i0 + r0) * K + (idx < U * K ? idx : 0)];
            }
        }
    };
    double ta[U][V], tb[U][V];
    double ca[NCV], cb2[NCV];
    int r = 0;
    // all rows dense; groups of U rows (nr is a multiple of U in the lab)
    load(ta, r);
    loadc(ca, r);
    while (true) {
        const bool nb = r + U < nr;
        load(tb, nb ? r + U : r);
        loadc(cb2, nb ? r + U : r);
        __builtin_amdgcn_sched_barrier(0);
        group(ta, r, ca);
        r += U;
        if (!nb) break;
        const bool na = r + U < nr;
        load(ta, na ? r + U : r);
        loadc(ca, na ? r + U : r);
        __builtin_amdgcn_sched_barrier(0);
        group(tb, r, cb2);
        r += U;
        if (!na) break;
    }
}


// Streaming-structure probe: the pass's memory traffic with no arithmetic.  U rows per
// iteration (all loads, then all stores), band of rb rows, 512-column tiles (2 doubles
// per lane), grid (tile, band); dynamic LDS caps workgroups per CU.
template <int U>
__global__ __launch_bounds__(256) void copy_kernel(double* __restrict__ T, int64_t ld, int64_t rows,
                                                   int64_t width, int rb) {
    extern __shared__ double dyn_lds[];
    const int64_t j = (int64_t)blockIdx.x * 512 + threadIdx.x * 2;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - 2;
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    if (rb < 0) dyn_lds[threadIdx.x] = 0.0;   // keeps the dynamic allocation
    for (int64_t i = i0; i < iend; i += U) {
        d2 t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = ldv<true>(T + (i + u) * ld + jc);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            t[u].x += 0.0;
            if (colok) stv<true>(T + (i + u) * ld + j, t[u]);
        }
    }
}


// Out-of-place streaming probe in form 21's shape (T -> To, one double per lane, U = 2 rows per
// iteration, next group loaded before this one is stored): NTH lanes per workgroup (256 = form 21;
// 768 = 12 waves, the most that 3 waves/SIMD of a 160-VGPR kernel allow), band of rb rows.
// Asks whether wider row segments per workgroup (6 KB instead of 2 KB) keep tall bands streaming.
template <int NTH>
__global__ __launch_bounds__(NTH) void copyw_kernel(const double* __restrict__ T, double* __restrict__ To,
                                                    int64_t ld, int64_t rows, int64_t width, int rb) {
    const int64_t j = (int64_t)blockIdx.x * NTH + threadIdx.x;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - 1;
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    double a0 = __builtin_nontemporal_load(T + i0 * ld + jc);
    double a1 = i0 + 1 < iend ? __builtin_nontemporal_load(T + (i0 + 1) * ld + jc) : 0.0;
    for (int64_t i = i0; i < iend; i += 2) {
        double b0 = 0.0, b1 = 0.0;
        if (i + 2 < iend) b0 = __builtin_nontemporal_load(T + (i + 2) * ld + jc);
        if (i + 3 < iend) b1 = __builtin_nontemporal_load(T + (i + 3) * ld + jc);
        if (colok) {
            __builtin_nontemporal_store(a0 + 0.0, To + i * ld + j);
            if (i + 1 < iend) __builtin_nontemporal_store(a1 + 0.0, To + (i + 1) * ld + j);
        }
        a0 = b0;
        a1 = b1;
    }
}

// Persistent interleaved probe: G workgroups per 512-column tile, workgroup (x, g) walks
// bands g, g + G, g + 2G, ... of rb rows; TF: grid x = tile (tile fastest) or band group.
template <int U>
__global__ __launch_bounds__(256) void copyp_kernel(double* __restrict__ T, int64_t ld, int64_t rows,
                                                    int64_t width, int rb, int G, int tf) {
    extern __shared__ double dyn_lds[];
    const int ntile = (int)((width + 511) / 512);
    const int x = tf ? blockIdx.x % ntile : blockIdx.x / G;
    const int g = tf ? blockIdx.x / ntile : blockIdx.x % G;
    const int64_t j = (int64_t)x * 512 + threadIdx.x * 2;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - 2;
    if (rb < 0) dyn_lds[threadIdx.x] = 0.0;
    for (int64_t i0 = (int64_t)g * rb; i0 < rows; i0 += (int64_t)G * rb) {
        const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
        for (int64_t i = i0; i < iend; i += U) {
            d2 t[U];
#pragma unroll
            for (int u = 0; u < U; ++u) t[u] = ldv<true>(T + (i + u) * ld + jc);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                t[u].x += 0.0;
                if (colok) stv<true>(T + (i + u) * ld + j, t[u]);
            }
        }
    }
}


// ---- coefficients in VGPRs, delivered by DPP row broadcast (row_newbcast:n: lane n of
// each 16-lane row to the whole row).  A coefficient register pair holds 16 coefficients
// (replicated over the 4 rows of the wave), loaded with one vector load per 16.
template <int N>
__device__ inline double bc_mov(double v) {
    return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + N, 0xf, 0xf, false);
}
__device__ inline double bcn(double v, int n) {
    switch (n) {
        case 0: return bc_mov<0>(v);   case 1: return bc_mov<1>(v);   case 2: return bc_mov<2>(v);
        case 3: return bc_mov<3>(v);   case 4: return bc_mov<4>(v);   case 5: return bc_mov<5>(v);
        case 6: return bc_mov<6>(v);   case 7: return bc_mov<7>(v);   case 8: return bc_mov<8>(v);
        case 9: return bc_mov<9>(v);   case 10: return bc_mov<10>(v); case 11: return bc_mov<11>(v);
        case 12: return bc_mov<12>(v); case 13: return bc_mov<13>(v); case 14: return bc_mov<14>(v);
        default: return bc_mov<15>(v);
    }
}
// t = fma(-c[lane n of the row], p, t) in one instruction
template <int N>
__device__ inline void fmac_bc(double& t, double c, double p) {
    asm("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf" : "+v"(t) : "v"(c), "v"(p), "n"(N));
}
__device__ inline void fmac_bcn(double& t, double c, double p, int n) {
    switch (n) {
        case 0: fmac_bc<0>(t, c, p); break;   case 1: fmac_bc<1>(t, c, p); break;
        case 2: fmac_bc<2>(t, c, p); break;   case 3: fmac_bc<3>(t, c, p); break;
        case 4: fmac_bc<4>(t, c, p); break;   case 5: fmac_bc<5>(t, c, p); break;
        case 6: fmac_bc<6>(t, c, p); break;   case 7: fmac_bc<7>(t, c, p); break;
        case 8: fmac_bc<8>(t, c, p); break;   case 9: fmac_bc<9>(t, c, p); break;
        case 10: fmac_bc<10>(t, c, p); break; case 11: fmac_bc<11>(t, c, p); break;
        case 12: fmac_bc<12>(t, c, p); break; case 13: fmac_bc<13>(t, c, p); break;
        case 14: fmac_bc<14>(t, c, p); break; default: fmac_bc<15>(t, c, p); break;
    }
}


// step I of a group's chain: l = I / U, u = I % U (all U rows at step l, then step l + 1)
template <int K, int V, int U, bool ASM, int I>
__device__ __forceinline__ void dstep(double (&t)[U][V], const double (&c)[U * K / 16], const double (&pr)[K][V]) {
    constexpr int l = I / U, u = I % U, idx = u * K + l;
    if constexpr (ASM) {
        fmac_bc<idx & 15>(t[u][0], c[idx >> 4], pr[l][0]);
        if constexpr (V == 2) fmac_bc<idx & 15>(t[u][1], c[idx >> 4], pr[l][1]);
    } else {
        const double f = bc_mov<idx & 15>(c[idx >> 4]);
        t[u][0] = __builtin_fma(-f, pr[l][0], t[u][0]);
        if constexpr (V == 2) t[u][1] = __builtin_fma(-f, pr[l][1], t[u][1]);
    }
}
template <int K, int V, int U, bool ASM, int... I>
__device__ __forceinline__ void dchain(double (&t)[U][V], const double (&c)[U * K / 16], const double (&pr)[K][V],
                                       std::integer_sequence<int, I...>) {
    (dstep<K, V, U, ASM, I>(t, c, pr), ...);
}

// f4 structure (P[0..K)[V] in VGPRs, groups of U rows, 256-row band) with the coefficients
// of the next group loaded with its rows; ASM: fused v_fmac_f64_dpp, else mov_dpp + fma.
template <bool NT, int K, int V, int U, bool ASM, int W = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) void f4d_kernel(const double* __restrict__ T, double* __restrict__ To,
                                                  int64_t ld, int64_t rows, int64_t width,
                                                  const double* __restrict__ Cr, const double* __restrict__ P,
                                                  int rb) {
    const int64_t j = (int64_t)blockIdx.x * (256 * V) + threadIdx.x * V;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - V;
    double pr[K][V];
#pragma unroll
    for (int l = 0; l < K; ++l) {
        if constexpr (V == 2) {
            const d2 v = *(const d2*)(P + (int64_t)l * ld + jc);
            pr[l][0] = v.x;
            pr[l][1] = v.y;
        } else {
            pr[l][0] = P[(int64_t)l * ld + jc];
        }
    }
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    const int l16 = threadIdx.x & 15;
    constexpr int NC = U * K / 16;   // coefficient doubles per lane per group
    auto load = [&](double (&t)[U][V], double (&c)[NC], int r0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double* p = T + (i0 + r0 + u) * ld + jc;
            if constexpr (V == 2) {
                const d2 v = ldv<NT>(p);
                t[u][0] = v.x;
                t[u][1] = v.y;
            } else {
                t[u][0] = NT ? __builtin_nontemporal_load(p) : *p;
            }
        }
#pragma unroll
        for (int v = 0; v < NC; ++v) {
            const int idx = v * 16 + l16;
            c[v] = Cr[(i0 + r0 + idx / K) * K + idx % K];
        }
    };
    auto group = [&](double (&t)[U][V], const double (&c)[NC], int r0) {
        dchain<K, V, U, ASM>(t, c, pr, std::make_integer_sequence<int, K * U>{});
        if (colok)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                double* p = To + (i0 + r0 + u) * ld + j;
                if constexpr (V == 2) {
                    d2 v;
                    v.x = t[u][0];
                    v.y = t[u][1];
                    stv<NT>(p, v);
                } else {
                    if (NT) __builtin_nontemporal_store(t[u][0], p);
                    else *p = t[u][0];
                }
            }
    };
    double ta[U][V], tb[U][V], ca[NC], cb[NC];
    int r = 0;
    load(ta, ca, r);
    while (true) {
        const bool nb = r + U < nr;
        load(tb, cb, nb ? r + U : r);
        __builtin_amdgcn_sched_barrier(0);
        group(ta, ca, r);
        r += U;
        if (!nb) break;
        const bool na = r + U < nr;
        load(ta, ca, na ? r + U : r);
        __builtin_amdgcn_sched_barrier(0);
        group(tb, cb, r);
        r += U;
        if (!na) break;
    }
}

// VALU rate probe: 8 independent chains per lane, ITER x 8 steps each.
// MODE 0: v_fma_f64 with an SGPR coefficient, 1: v_fmac_f64_dpp (row_newbcast) with a VGPR
// coefficient, 2: v_fma_f64 with a VGPR coefficient.
template <int MODE>
__global__ __launch_bounds__(256) void valu_kernel(double* out, double cs, int iters) {
    double t[8], p[8];
    const double cv = cs + threadIdx.x * 1e-3;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        t[k] = threadIdx.x + k;
        p[k] = 1.0 + k * 1e-9;
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                if constexpr (MODE == 0) t[k] = __builtin_fma(-cs, p[s], t[k]);
                else if constexpr (MODE == 1) fmac_bc<3>(t[k], cv, p[s]);
                else t[k] = __builtin_fma(-cv, p[s], t[k]);
            }
    }
    double a = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) a += t[k];
    out[blockIdx.x * 256 + threadIdx.x] = a;
}

// Latency probe: NCH independent chains per lane; MODE 1: v_fmac_f64_dpp, 2: v_fma_f64 (VGPR c)
template <int MODE, int NCH>
__global__ __launch_bounds__(256) void lat_kernel(double* out, double cs, int iters) {
    double t[NCH], p[8];
    const double cv = cs + threadIdx.x * 1e-3;
#pragma unroll
    for (int k = 0; k < NCH; ++k) t[k] = threadIdx.x + k;
#pragma unroll
    for (int k = 0; k < 8; ++k) p[k] = 1.0 + k * 1e-9;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int k = 0; k < NCH; ++k) {
                if constexpr (MODE == 1) fmac_bc<3>(t[k], cv, p[s]);
                else asm("v_fma_f64 %0, -%1, %2, %0" : "+v"(t[k]) : "v"(cv), "v"(p[s]));
            }
    }
    double a = 0;
#pragma unroll
    for (int k = 0; k < NCH; ++k) a += t[k];
    out[blockIdx.x * 256 + threadIdx.x] = a;
}

struct Lab {
    int64_t rows, width, ld;
    double *T, *To, *Cr, *P;
};

typedef void (*Launch)(const Lab&, int K, int rb, hipStream_t);

template <int K, int V, int U, int MODE>
void launch_f4(const Lab& L, int, int rb, hipStream_t s) {
    dim3 grid((unsigned)((L.width + 256 * V - 1) / (256 * V)), (unsigned)((L.rows + rb - 1) / rb));
    f4_kernel<true, K, V, U, MODE><<<grid, 256, 0, s>>>(L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb, 0.5);
}


// Pipelined stages: workgroup = S x 256 lanes; stage s (waves 4s..4s+3) applies steps
// [s KS, (s+1) KS) to groups of U rows of a 512-column tile, holding its P slice in VGPRs
// and reading its coefficients by scalar loads (form 4's chunks); stage 0 loads rows from
// HBM (one group ahead), stage S-1 stores them, stages hand groups on through LDS slots
// (two per stage boundary).  Iteration k: stage s works on group k - s; one barrier per
// iteration (raw s_barrier: the row prefetch stays in flight across it).
template <bool NT, int KS, int S, int U, int D>
__global__ __launch_bounds__(256 * S) void pipe_kernel(const double* __restrict__ T, double* __restrict__ To,
                                                       int64_t ld, int64_t rows, int64_t width,
                                                       const double* __restrict__ Cr, const double* __restrict__ P,
                                                       int rb) {
    constexpr int K = KS * S;
    __shared__ d2 slot[(S > 1 ? S - 1 : 1)][2][U][256];
    const int st = S == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);   // stage (wave-uniform)
    const int tid = threadIdx.x & 255;
    const int64_t j = (int64_t)blockIdx.x * 512 + tid * 2;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - 2;
    double pr[KS][2];
#pragma unroll
    for (int l = 0; l < KS; ++l) {
        const d2 v = *(const d2*)(P + (int64_t)(st * KS + l) * ld + jc);
        pr[l][0] = v.x;
        pr[l][1] = v.y;
    }
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int ng = (int)((iend - i0) / U);   // the lab's bands are whole groups
    constexpr int LC = 16 / U;
    auto chain = [&](double (&t)[U][2], int g) {
        const cdptr cb = (cdptr)(Cr + (i0 + (int64_t)g * U) * K + st * KS);
        double fa[U][LC], fb[U][LC];
        auto fetch = [&](double (&f)[U][LC], int l0) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int l = 0; l < LC; ++l) f[u][l] = cb[u * K + l0 + l];
        };
        auto run = [&](const double (&f)[U][LC], int l0) {
#pragma unroll
            for (int l = 0; l < LC; ++l)
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    t[u][0] = __builtin_fma(-f[u][l], pr[l0 + l][0], t[u][0]);
                    t[u][1] = __builtin_fma(-f[u][l], pr[l0 + l][1], t[u][1]);
                }
        };
        fetch(fa, 0);
#pragma unroll
        for (int l0 = 0; l0 < KS; l0 += 2 * LC) {
            __builtin_amdgcn_s_waitcnt(0xC07F);
            if (l0 + LC < KS) fetch(fb, l0 + LC);
            __builtin_amdgcn_sched_barrier(0);
            run(fa, l0);
            __builtin_amdgcn_sched_barrier(0);
            if (l0 + LC < KS) {
                __builtin_amdgcn_s_waitcnt(0xC07F);
                if (l0 + 2 * LC < KS) fetch(fa, l0 + 2 * LC);
                __builtin_amdgcn_sched_barrier(0);
                run(fb, l0 + LC);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    };
    auto load = [&](double (&t)[U][2], int g) {
        const int gg = g < ng ? g : ng - 1;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const d2 v = ldv<NT>(T + (i0 + (int64_t)gg * U + u) * ld + jc);
            t[u][0] = v.x;
            t[u][1] = v.y;
        }
    };
    // stage 0 keeps D - 1 groups of rows in flight: group g lives in buf[g % D]
    double buf[D][U][2];
    if (st == 0)
#pragma unroll
        for (int d = 0; d < D - 1; ++d) load(buf[d], d);
    const int total = ng + S - 1;
    for (int k = 0; k < total; k += D) {
#pragma unroll
        for (int h = 0; h < D; ++h) {
            const int kk = k + h;
            double (&cur)[U][2] = buf[h];
            const int g = kk - st;
            if (kk < total && g >= 0 && g < ng) {
                if (st == 0) {
                    load(buf[(h + D - 1) % D], g + D - 1);
                } else {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const d2 v = slot[st - 1][g & 1][u][tid];
                        cur[u][0] = v.x;
                        cur[u][1] = v.y;
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                chain(cur, g);
                __builtin_amdgcn_sched_barrier(0);
                if (st == S - 1) {
                    if (colok)
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            d2 v;
                            v.x = cur[u][0];
                            v.y = cur[u][1];
                            stv<NT>(To + (i0 + (int64_t)g * U + u) * ld + j, v);
                        }
                } else {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        d2 v;
                        v.x = cur[u][0];
                        v.y = cur[u][1];
                        slot[st][g & 1][u][tid] = v;
                    }
                }
            }
            if (S > 1 && kk < total) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
    }
}

template <int KS, int S, int U, int D>
void launch_pipe(const Lab& L, int, int rb, hipStream_t s) {
    dim3 grid((unsigned)((L.width + 511) / 512), (unsigned)((L.rows + rb - 1) / rb));
    pipe_kernel<true, KS, S, U, D><<<grid, 256 * S, 0, s>>>(L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb);
}


template <int K, int V, int U, bool ASM, int W = 1>
void launch_f4d(const Lab& L, int, int rb, hipStream_t s) {
    dim3 grid((unsigned)((L.width + 256 * V - 1) / (256 * V)), (unsigned)((L.rows + rb - 1) / rb));
    f4d_kernel<true, K, V, U, ASM, W><<<grid, 256, 0, s>>>(L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb);
}

// K = 64, V = 1, U = 2 with 1.5 coefficient sets: a group's coefficient pairs 0,1,4,5 are
// steps 0..31 of its two rows, 2,3,6,7 steps 32..63.  Group g: issue the loads of its
// second half (into the pairs group g-1's second half used), then rows g+1; steps 0..31;
// issue the first half of g+1 (into the pairs just consumed); steps 32..63; store.
template <int K, int V, int U, int I0, bool ASM, int... I>
__device__ __forceinline__ void dchain_part(double (&t)[U][V], const double (&c)[U * K / 16],
                                            const double (&pr)[K][V], std::integer_sequence<int, I...>) {
    (dstep<K, V, U, ASM, I0 + I>(t, c, pr), ...);
}
template <bool NT, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) void f4e_kernel(
    const double* __restrict__ T, double* __restrict__ To, int64_t ld, int64_t rows, int64_t width,
    const double* __restrict__ Cr, const double* __restrict__ P, int rb) {
    constexpr int K = 64, V = 1, U = 2, NC = 8;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - 1;
    double pr[K][V];
#pragma unroll
    for (int l = 0; l < K; ++l) pr[l][0] = P[(int64_t)l * ld + jc];
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    const int l16 = threadIdx.x & 15;
    double c[NC];
    auto loadc = [&](int r0, int half) {   // half 0: pairs 0,1,4,5; 1: pairs 2,3,6,7
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int v = (w >> 1) * 4 + half * 2 + (w & 1);
            const int idx = v * 16 + l16;
            c[v] = Cr[(i0 + r0 + idx / K) * K + idx % K];
        }
    };
    auto loadt = [&](double (&t)[U][V], int r0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double* p = T + (i0 + r0 + u) * ld + jc;
            t[u][0] = NT ? __builtin_nontemporal_load(p) : *p;
        }
    };
    auto group = [&](double (&t)[U][V], double (&tn)[U][V], int r0, int rn, bool more) {
        loadc(r0, 1);
        __builtin_amdgcn_sched_barrier(0);   // in-order vmcnt: the coefficients first
        loadt(tn, rn);
        __builtin_amdgcn_sched_barrier(0);
        dchain_part<K, V, U, 0, true>(t, c, pr, std::make_integer_sequence<int, K * U / 2>{});
        __builtin_amdgcn_sched_barrier(0);
        loadc(rn, 0);
        __builtin_amdgcn_sched_barrier(0);
        dchain_part<K, V, U, K * U / 2, true>(t, c, pr, std::make_integer_sequence<int, K * U / 2>{});
        if (colok)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                double* p = To + (i0 + r0 + u) * ld + j;
                if (NT) __builtin_nontemporal_store(t[u][0], p);
                else *p = t[u][0];
            }
    };
    double ta[U][V], tb[U][V];
    int r = 0;
    loadt(ta, 0);
    loadc(0, 0);
    while (true) {
        const bool nb = r + U < nr;
        group(ta, tb, r, nb ? r + U : r, nb);
        r += U;
        if (!nb) break;
        const bool na = r + U < nr;
        group(tb, ta, r, na ? r + U : r, na);
        r += U;
        if (!na) break;
    }
}
template <int W>
void launch_f4e(const Lab& L, int, int rb, hipStream_t s) {
    dim3 grid((unsigned)((L.width + 255) / 256), (unsigned)((L.rows + rb - 1) / rb));
    f4e_kernel<true, W><<<grid, 256, 0, s>>>(L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb);
}

// f4e with buffer loads/stores: band resources in SGPRs, one 32-bit column offset per lane
// (rows: soffset = row offset in the band; coefficients: C row-major, (u, l) at r0 K + u K + l).
template <bool NT, int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) void f4b_kernel(
    const double* __restrict__ T, double* __restrict__ To, int64_t ld, int64_t rows, int64_t width,
    const double* __restrict__ Cr, const double* __restrict__ P, int rb) {
    constexpr int K = 64, V = 1, U = 2, NC = 8;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool colok = j < width;
    const int jc = (int)(colok ? j : width - 1);
    double pr[K][V];
#pragma unroll
    for (int l = 0; l < K; ++l) pr[l][0] = P[(int64_t)l * ld + jc];
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(T + i0 * ld), (short)0, (int)((int64_t)nr * ld * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(To + i0 * ld), (short)0, colok ? (int)((int64_t)nr * ld * 8) : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Cr + i0 * K), (short)0, (int)((int64_t)nr * K * 8), 0x00020000);
    const int voff = jc * 8;
    const int coff = (threadIdx.x & 15) * 8;
    const int rowb = (int)(ld * 8);
    double c[NC];
    auto loadc = [&](int r0, int half) {   // half 0: pairs 0,1,4,5; 1: pairs 2,3,6,7
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int v = (w >> 1) * 4 + half * 2 + (w & 1);
            const u2v x = __builtin_amdgcn_raw_buffer_load_b64(rc, coff + v * 128, r0 * K * 8, 0);
            c[v] = __builtin_bit_cast(double, x);
        }
    };
    auto loadt = [&](double (&t)[U][V], int r0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u2v x = __builtin_amdgcn_raw_buffer_load_b64(rt, voff, (r0 + u) * rowb, NT ? 2 : 0);
            t[u][0] = __builtin_bit_cast(double, x);
        }
    };
    auto group = [&](double (&t)[U][V], double (&tn)[U][V], int r0, int rn) {
        loadc(r0, 1);
        __builtin_amdgcn_sched_barrier(0);   // in-order vmcnt: the coefficients first
        loadt(tn, rn);
        __builtin_amdgcn_sched_barrier(0);
        dchain_part<K, V, U, 0, true>(t, c, pr, std::make_integer_sequence<int, K * U / 2>{});
        __builtin_amdgcn_sched_barrier(0);
        loadc(rn, 0);
        __builtin_amdgcn_sched_barrier(0);
        dchain_part<K, V, U, K * U / 2, true>(t, c, pr, std::make_integer_sequence<int, K * U / 2>{});
#pragma unroll
        for (int u = 0; u < U; ++u)   // out-of-range lanes: num_records 0 drops the store
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, t[u][0]), ro, voff, (r0 + u) * rowb,
                                                  NT ? 2 : 0);
    };
    double ta[U][V], tb[U][V];
    int r = 0;
    loadt(ta, 0);
    loadc(0, 0);
    while (true) {
        const bool nb = r + U < nr;
        group(ta, tb, r, nb ? r + U : r);
        r += U;
        if (!nb) break;
        const bool na = r + U < nr;
        group(tb, ta, r, na ? r + U : r);
        r += U;
        if (!na) break;
    }
}
template <int W>
void launch_f4b(const Lab& L, int, int rb, hipStream_t s) {
    dim3 grid((unsigned)((L.width + 255) / 256), (unsigned)((L.rows + rb - 1) / rb));
    f4b_kernel<true, W><<<grid, 256, 0, s>>>(L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb);
}

// K = 64, V = 1, U rows, coefficients rolled by quarters: pair u*4 + q holds row u's steps
// [16q, 16q + 16); once quarter q of group g has run, those U pairs are reloaded with group
// g+1's quarter q.  Rows of g+1 are issued at the start of g, after every coefficient load
// group g still waits for.
template <int K, int V, int U, int Q, bool ASM, int... I>
__device__ __forceinline__ void qchain(double (&t)[U][V], const double (&c)[U * K / 16], const double (&pr)[K][V],
                                       std::integer_sequence<int, I...>) {
    // I enumerates (l within the quarter) * U + u
    (dstep<K, V, U, ASM, (Q * 16 + I / U) * U + I % U>(t, c, pr), ...);
}
template <bool NT, int U, int W, int CL = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) void f4q_kernel(
    const double* __restrict__ T, double* __restrict__ To, int64_t ld, int64_t rows, int64_t width,
    const double* __restrict__ Cr, const double* __restrict__ P, int rb) {
    constexpr int K = 64, V = 1, NC = U * 4;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool colok = j < width;
    const int jc = (int)(colok ? j : width - 1);
    double pr[K][V];
#pragma unroll
    for (int l = 0; l < K; ++l) pr[l][0] = P[(int64_t)l * ld + jc];
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(T + i0 * ld), (short)0, (int)((int64_t)nr * ld * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(To + i0 * ld), (short)0, colok ? (int)((int64_t)nr * ld * 8) : 0, 0x00020000);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Cr + i0 * K), (short)0, (int)((int64_t)nr * K * 8), 0x00020000);
    const int voff = jc * 8;
    const int coff = (threadIdx.x & 15) * 8;
    const int rowb = (int)(ld * 8);
    double c[NC];
    auto loadq = [&](int r0, int q) {
        if constexpr (CL == 1) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const u2v x = __builtin_amdgcn_raw_buffer_load_b64(rc, coff + (u * 4 + q) * 128, r0 * K * 8, 0);
                c[u * 4 + q] = __builtin_bit_cast(double, x);
            }
        } else if constexpr (CL == 2) {
            // quarter q of rows u, u+1 in one b128 per lane (timing only: wrong pairing)
#pragma unroll
            for (int u = 0; u < U; u += 2) {
                const u4v x = __builtin_amdgcn_raw_buffer_load_b128(rc, coff * 2 + (u * 4 + q) * 128, r0 * K * 8, 0);
                const d2 d = __builtin_bit_cast(d2, x);
                c[u * 4 + q] = d.x;
                c[(u + 1) * 4 + q] = d.y;
            }
        }
    };
    auto loadt = [&](double (&t)[U][V], int r0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u2v x = __builtin_amdgcn_raw_buffer_load_b64(rt, voff, (r0 + u) * rowb, NT ? 2 : 0);
            t[u][0] = __builtin_bit_cast(double, x);
        }
    };
    auto group = [&](double (&t)[U][V], double (&tn)[U][V], int r0, int rn) {
        loadt(tn, rn);
        __builtin_amdgcn_sched_barrier(0);
        qchain<K, V, U, 0, true>(t, c, pr, std::make_integer_sequence<int, 16 * U>{});
        __builtin_amdgcn_sched_barrier(0);
        loadq(rn, 0);
        __builtin_amdgcn_sched_barrier(0);
        qchain<K, V, U, 1, true>(t, c, pr, std::make_integer_sequence<int, 16 * U>{});
        __builtin_amdgcn_sched_barrier(0);
        loadq(rn, 1);
        __builtin_amdgcn_sched_barrier(0);
        qchain<K, V, U, 2, true>(t, c, pr, std::make_integer_sequence<int, 16 * U>{});
        __builtin_amdgcn_sched_barrier(0);
        loadq(rn, 2);
        __builtin_amdgcn_sched_barrier(0);
        qchain<K, V, U, 3, true>(t, c, pr, std::make_integer_sequence<int, 16 * U>{});
        __builtin_amdgcn_sched_barrier(0);
        loadq(rn, 3);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, t[u][0]), ro, voff, (r0 + u) * rowb,
                                                  NT ? 2 : 0);
    };
    double ta[U][V], tb[U][V];
    int r = 0;
    loadt(ta, 0);
#pragma unroll
    for (int q = 0; q < 4; ++q) loadq(0, q);
    while (true) {
        const bool nb = r + U < nr;
        group(ta, tb, r, nb ? r + U : r);
        r += U;
        if (!nb) break;
        const bool na = r + U < nr;
        group(tb, ta, r, na ? r + U : r);
        r += U;
        if (!na) break;
    }
}
template <int U, int W, int CL = 1>
void launch_f4q(const Lab& L, int, int rb, hipStream_t s) {
    dim3 grid((unsigned)((L.width + 255) / 256), (unsigned)((L.rows + rb - 1) / rb));
    f4q_kernel<true, U, W, CL><<<grid, 256, 0, s>>>(L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb);
}

// Pipelined stages with DPP coefficients: stage s (waves 4s..4s+3) applies steps
// [32 s, 32 s + 32) with its P slice (32 x 2 columns) in VGPRs; a row's 32 coefficients of
// the stage are ONE 16-B load per lane (lane n of each 16-lane row: steps 2n, 2n+1);
// stage 0 loads rows from HBM, stage S-1 stores, groups handed on through LDS slots.
template <int U, int... I>
__device__ __forceinline__ void pstep_all(double (&t)[U][2], const double (&c)[U][2], const double (&pr)[32][2],
                                          std::integer_sequence<int, I...>) {
    // I = m * U + u: step m of the stage for row u
    ((fmac_bc<((I / U) >> 1)>(t[I % U][0], c[I % U][(I / U) & 1], pr[I / U][0]),
      fmac_bc<((I / U) >> 1)>(t[I % U][1], c[I % U][(I / U) & 1], pr[I / U][1])), ...);
}
template <bool NT, int S, int U>
__global__ __launch_bounds__(256 * S) void piped_kernel(const double* __restrict__ T, double* __restrict__ To,
                                                        int64_t ld, int64_t rows, int64_t width,
                                                        const double* __restrict__ Cr, const double* __restrict__ P,
                                                        int rb) {
    constexpr int K = 32 * S;
    __shared__ d2 slot[(S > 1 ? S - 1 : 1)][2][U][256];
    const int st = S == 1 ? 0 : __builtin_amdgcn_readfirstlane(threadIdx.x >> 8);
    const int tid = threadIdx.x & 255;
    const int64_t j = (int64_t)blockIdx.x * 512 + tid * 2;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - 2;
    double pr[32][2];
#pragma unroll
    for (int l = 0; l < 32; ++l) {
        const d2 v = *(const d2*)(P + (int64_t)(st * 32 + l) * ld + jc);
        pr[l][0] = v.x;
        pr[l][1] = v.y;
    }
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int ng = (int)((iend - i0) / U);
    const int n16 = threadIdx.x & 15;
    auto loadc = [&](double (&c)[U][2], int g) {
        const int gg = g < ng ? g : ng - 1;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const d2 v = *(const d2*)(Cr + (i0 + (int64_t)gg * U + u) * K + st * 32 + 2 * n16);
            c[u][0] = v.x;
            c[u][1] = v.y;
        }
    };
    auto load = [&](double (&t)[U][2], int g) {
        const int gg = g < ng ? g : ng - 1;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const d2 v = ldv<NT>(T + (i0 + (int64_t)gg * U + u) * ld + jc);
            t[u][0] = v.x;
            t[u][1] = v.y;
        }
    };
    double ta[U][2], tb[U][2], ca[U][2], cb[U][2];
    if (st == 0) load(ta, 0);
    loadc(ca, 0 - 0);   // this stage's first group is g = 0 (reached at iteration st)
    const int total = ng + S - 1;
    for (int k = 0; k < total; k += 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kk = k + h;
            double (&cur)[U][2] = h == 0 ? ta : tb;
            double (&nxt)[U][2] = h == 0 ? tb : ta;
            double (&cc)[U][2] = h == 0 ? ca : cb;
            double (&cn)[U][2] = h == 0 ? cb : ca;
            const int g = kk - st;
            if (kk < total && g >= 0 && g < ng) {
                if (st == 0) load(nxt, g + 1);
                loadc(cn, g + 1);
                if (st > 0) {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const d2 v = slot[st - 1][g & 1][u][tid];
                        cur[u][0] = v.x;
                        cur[u][1] = v.y;
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                pstep_all<U>(cur, cc, pr, std::make_integer_sequence<int, 32 * U>{});
                __builtin_amdgcn_sched_barrier(0);
                if (st == S - 1) {
                    if (colok)
#pragma unroll
                        for (int u = 0; u < U; ++u) {
                            d2 v;
                            v.x = cur[u][0];
                            v.y = cur[u][1];
                            stv<NT>(To + (i0 + (int64_t)g * U + u) * ld + j, v);
                        }
                } else {
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        d2 v;
                        v.x = cur[u][0];
                        v.y = cur[u][1];
                        slot[st][g & 1][u][tid] = v;
                    }
                }
            } else if (kk < total && g < 0) {
                // stages > 0 idle until their first group; keep the coefficient ping-pong aligned
#pragma unroll
                for (int u = 0; u < U; ++u) { cn[u][0] = cc[u][0]; cn[u][1] = cc[u][1]; }
            }
            if (S > 1 && kk < total) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
    }
}
template <int S, int U>
void launch_piped(const Lab& L, int, int rb, hipStream_t s) {
    dim3 grid((unsigned)((L.width + 511) / 512), (unsigned)((L.rows + rb - 1) / rb));
    piped_kernel<true, S, U><<<grid, 256 * S, 0, s>>>(L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb);
}

// MFMA pass (v_mfma_f64_16x16x4f64 rounds as four sequential fmas in k order:
// tools/mfma_probe.hip).  Workgroup = 4 waves on one tile of 16*NT columns; the tile's
// P slab [K][16 NT] in LDS; wave w takes 16-row groups w, w+4, ... of the band.  Per
// group: acc tiles = T (accumulator layout: lane l, reg i -> row l/16 + 4i, column l%16),
// then for kblock b (steps 4b..4b+3) and tile t: acc[t] = mfma(-C frag, P frag, acc[t]).
// Coefficients are read in the permuted layout Cm[row][q*(K/4) + b] = C[row][4b + q] so
// that lane (r = l%16, q = l/16) reads its K/4 values contiguously.
typedef double d4 __attribute__((ext_vector_type(4)));
template <int K, int NT>
__global__ __launch_bounds__(256) void mpass_kernel(const double* __restrict__ T, double* __restrict__ To,
                                                    int64_t ld, int64_t rows, int64_t width,
                                                    const double* __restrict__ Cm, const double* __restrict__ P,
                                                    int rb) {
    constexpr int W = 16 * NT, KB = K / 4;
    __shared__ double Ps[K * W];
    const int64_t c0 = (int64_t)blockIdx.x * W;
    for (int e = threadIdx.x; e < K * W; e += 256) {
        const int l = e / W, c = e % W;
        const int64_t cc = c0 + c < width ? c0 + c : width - 1;
        Ps[e] = P[(int64_t)l * ld + cc];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int lr = lane & 15, lq = lane >> 4;
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int ng = (int)((iend - i0) / 16);
    for (int g = w; g < ng; g += 4) {
        const int64_t r0 = i0 + (int64_t)g * 16;
        d4 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int64_t col = c0 + 16 * t + lr;
            const int64_t cc = col < width ? col : width - 1;
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[t][i] = __builtin_nontemporal_load(T + (r0 + lq + 4 * i) * ld + cc);
        }
        double a[KB];
        const double* cp = Cm + (r0 + lr) * K + lq * KB;
#pragma unroll
        for (int b = 0; b < KB; b += 2) {
            const d2 v = *(const d2*)(cp + b);
            a[b] = -v.x;
            a[b + 1] = -v.y;
        }
#pragma unroll
        for (int b = 0; b < KB; ++b) {
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const double bv = Ps[(4 * b + lq) * W + 16 * t + lr];
                acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[b], bv, acc[t], 0, 0, 0);
            }
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int64_t col = c0 + 16 * t + lr;
            if (col < width)
#pragma unroll
                for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(acc[t][i], To + (r0 + lq + 4 * i) * ld + col);
        }
    }
}
template <int K, int NT>
void launch_mpass(const Lab& L, int, int rb, hipStream_t s) {
    dim3 grid((unsigned)((L.width + 16 * NT - 1) / (16 * NT)), (unsigned)((L.rows + rb - 1) / rb));
    mpass_kernel<K, NT><<<grid, 256, 0, s>>>(L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb);
}
// reference for the permuted coefficient layout
__global__ void ref_m_kernel(const double* T, double* To, int64_t ld, int64_t rows, int64_t width, int K,
                             const double* Cm, const double* P) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t i = blockIdx.y;
    if (j >= width || i >= rows) return;
    const int KB = K / 4;
    double t = T[i * ld + j];
    for (int l = 0; l < K; ++l) t = __builtin_fma(-Cm[i * K + (l % 4) * KB + l / 4], P[(int64_t)l * ld + j], t);
    To[i * ld + j] = t;
}

// MFMA pass v2: the 4 waves of a workgroup share each 16-row group and take NT 16-column
// tiles each (workgroup = 64 NT columns); P fragments (K/4 x NT doubles per lane) stay in
// registers for the band; the group's coefficient rows (Cm, 16 x K doubles, contiguous) are
// staged in LDS by LDS-DMA one group ahead (double buffer, rows padded by PAD doubles); the
// next group's T tile is prefetched into registers.
template <int K, int NT, int PAD>
__global__ __launch_bounds__(256, 2) void mpass2_kernel(const double* __restrict__ T, double* __restrict__ To,
                                                       int64_t ld, int64_t rows, int64_t width,
                                                       const double* __restrict__ Cm, const double* __restrict__ P,
                                                       int rb) {
    constexpr int KB = K / 4, W = 16 * NT, RS = K + PAD;
    __shared__ double As[2][16 * RS];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lr = lane & 15, lq = lane >> 4;
    const int64_t c0 = (int64_t)blockIdx.x * (4 * W) + w * W;
    double b[KB][NT];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int64_t col = c0 + 16 * t + lr;
            b[kb][t] = P[(int64_t)(4 * kb + lq) * ld + (col < width ? col : width - 1)];
        }
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int ng = (int)((iend - i0) / 16);
    // stage the coefficients of group g into buffer g & 1: 16 rows of K doubles (K * 8 / 1024
    // wave instructions per row), rows spread over the 4 waves
    auto stage = [&](int g) {
        const int gg = g < ng ? g : ng - 1;
        const double* src = Cm + (i0 + (int64_t)gg * 16) * K;
        constexpr int PER_ROW = K * 8 / 1024;   // 1 KiB pieces per row (K = 128: 1)
        for (int pc = w; pc < 16 * PER_ROW; pc += 4) {
            const int r = pc / PER_ROW, part = pc % PER_ROW;
            __builtin_amdgcn_global_load_lds(src + r * K + part * 128 + lane * 2,
                                             (__attribute__((address_space(3))) void*)&As[g & 1][r * RS + part * 128],
                                             16, 0, 0);
        }
    };
    auto loadt = [&](d4 (&acc)[NT], int g) {
        const int gg = g < ng ? g : ng - 1;
        const int64_t r0 = i0 + (int64_t)gg * 16;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int64_t col = c0 + 16 * t + lr;
            const int64_t cc = col < width ? col : width - 1;
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[t][i] = __builtin_nontemporal_load(T + (r0 + lq + 4 * i) * ld + cc);
        }
    };
    d4 ta[NT], tb[NT];
    stage(0);
    loadt(ta, 0);
    for (int g = 0; g < ng; g += 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int gg = g + h;
            if (gg >= ng) break;
            d4 (&acc)[NT] = h == 0 ? ta : tb;
            d4 (&nxt)[NT] = h == 0 ? tb : ta;
            __syncthreads();   // everyone is done with buffer (gg + 1) & 1 (group gg - 1)
            stage(gg + 1);
            loadt(nxt, gg + 1);
            // wait for this group's coefficients (and its T tile): everything but the loads just issued
            constexpr int NEWV = NT * 4 + (K * 8 / 1024 * 16 + 3) / 4;
            __builtin_amdgcn_s_waitcnt(0x3F70 | (NEWV & 0xF) | ((NEWV >> 4) << 14));
            __syncthreads();
            const double* a = &As[gg & 1][lr * RS + lq * KB];
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                const double av = -a[kb];
#pragma unroll
                for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b[kb][t], acc[t], 0, 0, 0);
            }
            const int64_t r0 = i0 + (int64_t)gg * 16;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int64_t col = c0 + 16 * t + lr;
                if (col < width)
#pragma unroll
                    for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(acc[t][i], To + (r0 + lq + 4 * i) * ld + col);
            }
        }
    }
}
template <int K, int NT, int PAD>
void launch_mpass2(const Lab& L, int, int rb, hipStream_t s) {
    dim3 grid((unsigned)((L.width + 64 * NT - 1) / (64 * NT)), (unsigned)((L.rows + rb - 1) / rb));
    mpass2_kernel<K, NT, PAD><<<grid, 256, 0, s>>>(L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb);
}

// MFMA pass v3: as v2 with the coefficients staged 2 groups ahead in a 3-buffer LDS ring
// and the T tiles prefetched 2 groups ahead in a 3-deep register ring: one barrier per group.
template <int K, int NT, int PAD>
__global__ __launch_bounds__(256, 2) void mpass3_kernel(const double* __restrict__ T, double* __restrict__ To,
                                                       int64_t ld, int64_t rows, int64_t width,
                                                       const double* __restrict__ Cm, const double* __restrict__ P,
                                                       int rb) {
    constexpr int KB = K / 4, W = 16 * NT, RS = K + PAD;
    __shared__ double As[3][16 * RS];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lr = lane & 15, lq = lane >> 4;
    const int64_t c0 = (int64_t)blockIdx.x * (4 * W) + w * W;
    double b[KB][NT];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int64_t col = c0 + 16 * t + lr;
            b[kb][t] = P[(int64_t)(4 * kb + lq) * ld + (col < width ? col : width - 1)];
        }
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int ng = (int)((iend - i0) / 16);
    constexpr int PER_ROW = K * 8 / 1024;
    constexpr int STG = (16 * PER_ROW + 3) / 4;   // staging instructions per wave per group
    auto stage = [&](int g, int buf) {
        const int gg = g < ng ? g : ng - 1;
        const double* src = Cm + (i0 + (int64_t)gg * 16) * K;
        for (int pc = w; pc < 16 * PER_ROW; pc += 4) {
            const int r = pc / PER_ROW, part = pc % PER_ROW;
            __builtin_amdgcn_global_load_lds(src + r * K + part * 128 + lane * 2,
                                             (__attribute__((address_space(3))) void*)&As[buf][r * RS + part * 128],
                                             16, 0, 0);
        }
    };
    auto loadt = [&](d4 (&acc)[NT], int g) {
        const int gg = g < ng ? g : ng - 1;
        const int64_t r0 = i0 + (int64_t)gg * 16;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int64_t col = c0 + 16 * t + lr;
            const int64_t cc = col < width ? col : width - 1;
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[t][i] = __builtin_nontemporal_load(T + (r0 + lq + 4 * i) * ld + cc);
        }
    };
    d4 tr[3][NT];
    stage(0, 0);
    loadt(tr[0], 0);
    stage(1, 1);
    loadt(tr[1], 1);
    for (int g = 0; g < ng; g += 3) {
#pragma unroll
        for (int h = 0; h < 3; ++h) {
            const int gg = g + h;
            if (gg >= ng) break;
            // this group's staging + tile: everything but the last group's issue (one group's
            // worth of loads) and its stores
            constexpr int NEWV = NT * 4 + STG + NT * 4;
            __builtin_amdgcn_s_waitcnt(0x3F70 | (NEWV & 0xF) | ((NEWV >> 4) << 14));
            __syncthreads();   // group gg's coefficients are in; group gg-1's buffer is free
            stage(gg + 2, (h + 2) % 3);
            loadt(tr[(h + 2) % 3], gg + 2);
            d4 (&acc)[NT] = tr[h];
            const double* a = &As[h][lr * RS + lq * KB];
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                const double av = -a[kb];
#pragma unroll
                for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b[kb][t], acc[t], 0, 0, 0);
            }
            const int64_t r0 = i0 + (int64_t)gg * 16;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int64_t col = c0 + 16 * t + lr;
                if (col < width)
#pragma unroll
                    for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(acc[t][i], To + (r0 + lq + 4 * i) * ld + col);
            }
        }
    }
}
template <int K, int NT, int PAD>
void launch_mpass3(const Lab& L, int, int rb, hipStream_t s) {
    dim3 grid((unsigned)((L.width + 64 * NT - 1) / (64 * NT)), (unsigned)((L.rows + rb - 1) / rb));
    mpass3_kernel<K, NT, PAD><<<grid, 256, 0, s>>>(L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb);
}

// MFMA pass v4 (the product candidate for K = 64): coefficients read row-major (C[row][l],
// ldc = K), staged per 16-row group into LDS rows padded to RS = K + 2 doubles by LDS-DMA
// with per-lane source addresses (the LDS side is lane-linear: lane L of piece q lands at
// linear double 128 q + 2 L, so the source is the (row, column) that position means in the
// padded layout); A fragment of lane (r, q) at kblock b = -As[r][4 b + q].  Coefficient
// staging and T tiles one group ahead (register ring of 2), NT 16-column tiles per wave.
template <int K, int NT, int WPE = 2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void mpass4_kernel(const double* __restrict__ T, double* __restrict__ To,
                                                       int64_t ld, int64_t rows, int64_t width,
                                                       const double* __restrict__ Cr, const double* __restrict__ P,
                                                       int rb) {
    constexpr int KB = K / 4, W = 16 * NT, RS = K + 2;
    constexpr int NPC = (16 * RS + 127) / 128;   // 1 KiB pieces per group
    __shared__ double As[2][NPC * 128];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lr = lane & 15, lq = lane >> 4;
    const int64_t c0 = (int64_t)blockIdx.x * (4 * W) + w * W;
    double b[KB][NT];
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int64_t col = c0 + 16 * t + lr;
            b[kb][t] = P[(int64_t)(4 * kb + lq) * ld + (col < width ? col : width - 1)];
        }
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    const int ng = (nr + 15) / 16;
    auto stage = [&](int g, int buf) {
        const int gg = g < ng ? g : ng - 1;
        for (int pc = w; pc < NPC; pc += 4) {
            const int e0 = pc * 128 + 2 * lane;
            int r = e0 / RS, c = e0 % RS;
            if (c >= K || r >= 16) { r = 0; c = 0; }   // padding: any valid source
            int64_t row = i0 + (int64_t)gg * 16 + r;
            row = row < iend ? row : iend - 1;
            __builtin_amdgcn_global_load_lds(Cr + row * K + c,
                                             (__attribute__((address_space(3))) void*)&As[buf][pc * 128], 16, 0, 0);
        }
    };
    auto loadt = [&](d4 (&acc)[NT], int g) {
        const int gg = g < ng ? g : ng - 1;
        const int64_t r0 = i0 + (int64_t)gg * 16;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int64_t col = c0 + 16 * t + lr;
            const int64_t cc = col < width ? col : width - 1;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int64_t row = r0 + lq + 4 * i;
                row = row < iend ? row : iend - 1;
                acc[t][i] = __builtin_nontemporal_load(T + row * ld + cc);
            }
        }
    };
    d4 ta[NT], tb[NT];
    stage(0, 0);
    loadt(ta, 0);
    constexpr int STG = (NPC + 3) / 4;
    for (int g = 0; g < ng; g += 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int gg = g + h;
            if (gg >= ng) break;
            d4 (&acc)[NT] = h == 0 ? ta : tb;
            d4 (&nxt)[NT] = h == 0 ? tb : ta;
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // raw: the prefetch stays in flight
            stage(gg + 1, (gg + 1) & 1);
            loadt(nxt, gg + 1);
            constexpr int NEWV = NT * 4 + STG;
            __builtin_amdgcn_s_waitcnt(0x3F70 | (NEWV & 0xF) | ((NEWV >> 4) << 14));
            asm volatile("s_barrier" ::: "memory");
            const double* a = &As[gg & 1][lr * RS + lq];
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) {
                const double av = -a[4 * kb];
#pragma unroll
                for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b[kb][t], acc[t], 0, 0, 0);
            }
            const int64_t r0 = i0 + (int64_t)gg * 16;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int64_t col = c0 + 16 * t + lr;
                if (col < width)
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        if (r0 + lq + 4 * i < iend)
                            __builtin_nontemporal_store(acc[t][i], To + (r0 + lq + 4 * i) * ld + col);
            }
        }
    }
}
template <int K, int NT, int W = 2>
void launch_mpass4(const Lab& L, int, int rb, hipStream_t s) {
    dim3 grid((unsigned)((L.width + 64 * NT - 1) / (64 * NT)), (unsigned)((L.rows + rb - 1) / rb));
    mpass4_kernel<K, NT, W><<<grid, 256, 0, s>>>(L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb);
}

// ---- f4r: form 21's compute (P[0..64) of one column per lane in VGPRs, 2 rows per
// group, coefficients broadcast by v_fmac_f64_dpp) with the rows AND the coefficient rows
// of each group staged per wave in an LDS ring of D groups by LDS-DMA
// (global_load_lds_dwordx4 from inline asm: the compiler does not count it, the kernel
// waits with its own counted vmcnt), so D groups of loads are in flight per wave instead
// of one group in registers.  Ring slot (2 KB): rows r0, r0+1 x the wave's 64 columns
// (lane l's 16 B = row l / 32, columns 2 (l % 32) .. +1), then the two rows' 64
// coefficients each (lane l: row l / 32, steps 2 (l % 32) .. +1).
__device__ __forceinline__ void glds16(const void* g, uint32_t m0) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}
template <int N>
__device__ __forceinline__ void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// newer than group g's U DMAs: U per prologue group still to come, 2 U (U stores + U DMAs)
// per finished group: U (D - 1) + U g while g < D - 1, then 2 U (D - 1)
template <int D, int U>
__device__ __forceinline__ void vmwait_group(int g) {
    if (g >= D - 1) { vmwait<2 * U * (D - 1)>(); return; }
    switch (g) {
        case 0: vmwait<U * (D - 1)>(); break;
        case 1: vmwait<U * (D - 1) + U>(); break;
        case 2: vmwait<U * (D - 1) + 2 * U>(); break;
        case 3: vmwait<U * (D - 1) + 3 * U>(); break;
        case 4: vmwait<U * (D - 1) + 4 * U>(); break;
        case 5: vmwait<U * (D - 1) + 5 * U>(); break;
        default: vmwait<U * (D - 1) + 6 * U>(); break;
    }
}
// step L of a half (coefficients of that half in c[u][even/odd]) for the U rows
template <int U, int L>
__device__ __forceinline__ void rstep(double (&t)[U], const double (&c)[U][2], const double (&pr)[64]) {
    constexpr int e = L & 1, n = (L & 31) >> 1;
#pragma unroll
    for (int u = 0; u < U; ++u) fmac_bc<n>(t[u], c[u][e], pr[L]);
}
template <int U, int L0, int... I>
__device__ __forceinline__ void rhalf(double (&t)[U], const double (&c)[U][2], const double (&pr)[64],
                                      std::integer_sequence<int, I...>) {
    (rstep<U, L0 + I>(t, c, pr), ...);
}
// ---- f4r: form 21's compute (P[0..64) of one column per lane in VGPRs, coefficients
// broadcast by v_fmac_f64_dpp) with the U rows AND their coefficient rows of each group
// staged per wave in an LDS ring of D groups by LDS-DMA (global_load_lds_dwordx4 from
// inline asm: the compiler does not count it; the kernel waits with its own counted vmcnt),
// so D groups of loads are in flight per wave instead of one group in registers.  Ring
// slot (1 KB per row): U rows x the wave's 64 columns (DMA k: rows 2k, 2k+1; lane l's 16 B
// = row 2k + l / 32, columns 2 (l % 32) .. +1), then the U rows' 64 coefficients (same
// layout).  The coefficients of one 32-step half at a time are in registers.
// MODE 0: the pass; 1: no fmas (the ring's streaming structure alone); 2: no memory in the
// loop (the first group's slot reused, no stores: the chain's compute alone; wrong values)
// IL: interleaved row groups instead of bands: workgroup (tile, gi), gi < G = gridDim.y, takes
// the U-row groups gi, gi + G, gi + 2G, ... of the whole height (P loaded once per
// workgroup; the resident workgroups' row fronts stay within ~G U rows of each other, as
// short bands' do)
template <bool NT, int U, int D, int W, int MODE = 0, bool IL = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(W))) void f4r_kernel(
    const double* __restrict__ T, double* __restrict__ To, int64_t ld, int64_t rows, int64_t width,
    const double* __restrict__ Cr, const double* __restrict__ P, int rb) {
    constexpr int K = 64, SLOT = 128 * U;   // doubles per ring slot
    extern __shared__ double ring[];   // [4 waves][D slots][SLOT]
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool colok = j < width;
    const int jc = (int)(colok ? j : width - 1);
    double pr[K];
#pragma unroll
    for (int l = 0; l < K; ++l) pr[l] = P[(int64_t)l * ld + jc];
    const int G = IL ? (int)gridDim.y : 1, gi = IL ? (int)blockIdx.y : 0;
    const int64_t i0 = IL ? 0 : (int64_t)blockIdx.y * rb;
    const int64_t iend = IL ? rows : ((i0 + rb < rows) ? i0 + rb : rows);
    const int nr = (int)(iend - i0);
    // groups of this workgroup (the lab's heights are multiples of U rows)
    const int ng = IL ? (int)((rows / U - gi + G - 1) / G) : nr / U;
    auto grow = [&](int g) -> int64_t { return IL ? ((int64_t)gi + (int64_t)G * g) * U : (int64_t)g * U; };
    const int64_t wc = (int64_t)blockIdx.x * 256 + w * 64 + 2 * (lane & 31);
    const int64_t wcc = wc < ld - 1 ? wc : ld - 2;
    const double* tsrc = T + (i0 + (lane >> 5)) * ld + wcc;
    const double* csrc = Cr + (i0 + (lane >> 5)) * K + 2 * (lane & 31);
    double* wbase = ring + (size_t)w * D * SLOT;
    const uint32_t lbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)wbase;
    const int voff = colok ? jc * 8 : 0x7fffff00;
    const int rowb = (int)(ld * 8);
    auto dma = [&](int g, int s) {
        const int64_t r = grow(g < ng ? g : ng - 1);
#pragma unroll
        for (int k = 0; k < U / 2; ++k)
            glds16(tsrc + (r + 2 * k) * ld, __builtin_amdgcn_readfirstlane(lbase + s * SLOT * 8 + k * 1024));
#pragma unroll
        for (int k = 0; k < U / 2; ++k)
            glds16(csrc + (r + 2 * k) * K,
                   __builtin_amdgcn_readfirstlane(lbase + s * SLOT * 8 + U * 512 + k * 1024));
    };
#pragma unroll
    for (int s = 0; s < D; ++s) dma(s, s);
    int s = 0;
    if (MODE == 2) vmwait<0>();
    for (int g = 0; g < ng; ++g) {
        if (MODE != 2) vmwait_group<D, U>(g);   // U DMA instructions per group (U / 2 row pairs, rows + coefficients)
        const double* sl = wbase + (MODE == 2 ? 0 : s) * SLOT;
        double t[U];
#pragma unroll
        for (int u = 0; u < U; ++u) t[u] = sl[u * 64 + lane];
        double c[U][2];
        auto loadc = [&](int h) {
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const d2 v = *(const d2*)(sl + U * 64 + u * 64 + h * 32 + 2 * (lane & 15));
                c[u][0] = v.x;
                c[u][1] = v.y;
            }
        };
        if constexpr (MODE != 1) {
            loadc(0);
            rhalf<U, 0>(t, c, pr, std::make_integer_sequence<int, 32>{});
            loadc(1);
            rhalf<U, 32>(t, c, pr, std::make_integer_sequence<int, 32>{});
        }
        if constexpr (MODE == 2) {
            if (t[0] == 12345.678) To[0] = t[1];   // keep the chains
            continue;
        }
        // a uniform descriptor per group (a per-lane one becomes a waterfall loop of stores,
        // which would break the counted waits); lanes past the width aim out of range
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(To + (i0 + grow(g)) * ld), (short)0, (int)((int64_t)U * ld * 8), 0x00020000);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double v = t[u];
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), ro, voff, u * rowb, NT ? 2 : 0);
        }
        dma(g + D, s);
        s = s + 1 == D ? 0 : s + 1;
    }
}
template <int U, int D, int W, int MODE = 0, int G = 0, bool NT = true>
void launch_f4r(const Lab& L, int, int rb, hipStream_t s) {
    if (G > 0) {   // interleaved: G workgroups per 256-column tile
        dim3 grid((unsigned)((L.width + 255) / 256), (unsigned)G);
        f4r_kernel<NT, U, D, W, MODE, true><<<grid, 256, (size_t)4 * D * 1024 * U, s>>>(
            L.T, L.To, L.ld, L.rows, L.width, L.Cr, L.P, rb);
        return;
    }
    dim3 grid((unsigned)((L.width + 255) / 256), (unsigned)((L.rows + rb - 1) / rb));
    f4r_kernel<NT, U, D, W, MODE><<<grid, 256, (size_t)4 * D * 1024 * U, s>>>(L.T, L.To, L.ld, L.rows, L.width,
                                                                               L.Cr, L.P, rb);
}

struct Variant {
    const char* name;
    int K, rb;
    Launch fn;
    bool exact;   // checked against the reference
    bool perm = false;   // coefficients in the MFMA-permuted layout
};

static bool check(const Variant& v) {
    Lab L;
    L.rows = 1024;
    L.width = 4112;   // 8 tiles of 512 + a ragged one
    L.ld = 4608;
    const int K = v.K;
    CK(hipMalloc(&L.T, L.rows * L.ld * 8));
    CK(hipMalloc(&L.To, L.rows * L.ld * 8));
    double* Tr;
    CK(hipMalloc(&Tr, L.rows * L.ld * 8));
    CK(hipMalloc(&L.Cr, L.rows * K * 8));
    CK(hipMalloc(&L.P, (int64_t)K * L.ld * 8));
    fill_kernel<<<1024, 256>>>(L.T, L.rows * L.ld, 1);
    fill_kernel<<<1024, 256>>>(L.Cr, L.rows * K, 2);
    fill_kernel<<<1024, 256>>>(L.P, (int64_t)K * L.ld, 3);
    CK(hipMemset(L.To, 0, L.rows * L.ld * 8));
    CK(hipMemset(Tr, 0, L.rows * L.ld * 8));
    if (v.perm)
        ref_m_kernel<<<dim3((unsigned)((L.width + 255) / 256), (unsigned)L.rows), 256>>>(L.T, Tr, L.ld, L.rows,
                                                                                        L.width, K, L.Cr, L.P);
    else
        ref_kernel<<<dim3((unsigned)((L.width + 255) / 256), (unsigned)L.rows), 256>>>(L.T, Tr, L.ld, L.rows, L.width,
                                                                                      K, L.Cr, L.P);
    v.fn(L, K, v.rb < L.rows ? v.rb : 256, 0);
    CK(hipDeviceSynchronize());
    std::vector<double> a(L.rows * L.ld), b(L.rows * L.ld);
    CK(hipMemcpy(a.data(), L.To, a.size() * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), Tr, b.size() * 8, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t i = 0; i < L.rows; ++i)
        for (int64_t jj = 0; jj < L.width; ++jj)
            if (memcmp(&a[i * L.ld + jj], &b[i * L.ld + jj], 8) != 0) ++bad;
    CK(hipFree(L.T));
    CK(hipFree(L.To));
    CK(hipFree(Tr));
    CK(hipFree(L.Cr));
    CK(hipFree(L.P));
    if (bad) printf("  CHECK %-28s K=%d: %ld of %ld elements differ\n", v.name, K, (long)bad,
                    (long)(L.rows * L.width));
    return bad == 0;
}

int main(int argc, char** argv) {
    const int64_t rows = argc > 1 ? atoll(argv[1]) : 32768;
    const int64_t ncols = argc > 2 ? atoll(argv[2]) : 65537;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    const char* only = argc > 4 ? argv[4] : nullptr;
    std::vector<Variant> vs = {
        // round 5: band counts against the 768 pass slots (257 tiles x 43 / 42 / 48 bands), the
        // interleaved persistent form on exactly 256 tiles (ncols 65536: G x 256 = 768 slots),
        // the MFMA pass at 3-4 waves per SIMD
        {"r5 f4r rb768", 64, 768, launch_f4r<4, 3, 3>, true},
        {"r5 f4r rb784", 64, 784, launch_f4r<4, 3, 3>, true},
        {"r5 f4r rb684", 64, 684, launch_f4r<4, 3, 3>, true},
        {"r5 f4r G3", 64, 768, launch_f4r<4, 3, 3, 0, 3>, true},
        {"r5 f4r G3 copy", 64, 768, launch_f4r<4, 3, 3, 1, 3>, false},
        {"r5 f4r G6", 64, 768, launch_f4r<4, 3, 3, 0, 6>, true},
        {"r5 f4r U2D4 G3", 64, 768, launch_f4r<2, 4, 3, 0, 3>, true},
        {"r5 mpass4 NT2 w4 rb768", 64, 768, launch_mpass4<64, 2, 4>, true},
        {"r5 mpass4 NT3 w3 rb768", 64, 768, launch_mpass4<64, 3, 3>, true},
        {"r5 mpass4 NT4 w2 rb768", 64, 768, launch_mpass4<64, 4, 2>, true},
        {"r5 mpass4 NT2 w4 rb256", 64, 256, launch_mpass4<64, 2, 4>, true},
        {"f4r K64 U4 D3 w3", 64, 768, launch_f4r<4, 3, 3>, true},
        {"f4r K64 U4 D3 w3 copy", 64, 768, launch_f4r<4, 3, 3, 1>, false},
        {"f4r K64 U4 D3 w3 nnt", 64, 768, launch_f4r<4, 3, 3, 0, 0, false>, true},
        {"f4r K64 U4 D3 w3 rb1536", 64, 1536, launch_f4r<4, 3, 3>, true},
        {"f4r K64 U2 D4 w3", 64, 768, launch_f4r<2, 4, 3>, true},
        {"f4q K64 V1U2 w3 rb768", 64, 768, launch_f4q<2, 3>, true},
        {"f4d K32 V2U2 mov", 32, 256, launch_f4d<32, 2, 2, false>, true},
        {"f4d K32 V2U2 asm", 32, 256, launch_f4d<32, 2, 2, true>, true},
        {"f4d K32 V2U4 asm", 32, 256, launch_f4d<32, 2, 4, true>, true},
        {"f4d K64 V1U2 mov", 64, 256, launch_f4d<64, 1, 2, false>, true},
        {"f4d K64 V1U2 asm", 64, 256, launch_f4d<64, 1, 2, true>, true},
        {"f4d K64 V1U4 asm", 64, 256, launch_f4d<64, 1, 4, true>, true},
        {"f4d K64 V1U8 asm", 64, 256, launch_f4d<64, 1, 8, true>, true},
        {"f4e K64 V1U2 w1", 64, 256, launch_f4e<1>, true},
        {"f4b K64 V1U2 w1", 64, 256, launch_f4b<1>, true},
        {"f4q K64 V1U2 w3", 64, 256, launch_f4q<2, 3>, true},
        {"mpass4 K64 NT4", 64, 256, launch_mpass4<64, 4>, true},
        {"mpass4 K64 NT4 rb512", 64, 512, launch_mpass4<64, 4>, true},
        {"mpass4 K64 NT2", 64, 256, launch_mpass4<64, 2>, true},
        {"mpass4 K64 NT4 rb250", 64, 250, launch_mpass4<64, 4>, true},
        {"mpass3 K128 NT2 p2", 128, 256, launch_mpass3<128, 2, 2>, true, true},
        {"mpass3 K128 NT2 p2 rb512", 128, 512, launch_mpass3<128, 2, 2>, true, true},
        {"mpass3 K128 NT2 p2 rb1008", 128, 1008, launch_mpass3<128, 2, 2>, true, true},
        {"mpass3 K128 NT1 p2 rb512", 128, 512, launch_mpass3<128, 1, 2>, true, true},
        {"mpass2 K128 NT2 p2", 128, 256, launch_mpass2<128, 2, 2>, true, true},
        {"mpass2 K128 NT2 p0", 128, 256, launch_mpass2<128, 2, 0>, true, true},
        {"mpass2 K128 NT1 p2", 128, 256, launch_mpass2<128, 1, 2>, true, true},
        {"mpass2 K64 NT4 p2", 64, 256, launch_mpass2<64, 4, 2>, true, true},
        {"mpass2 K128 NT2 p2 rb512", 128, 512, launch_mpass2<128, 2, 2>, true, true},
        {"mpass K64 NT4", 64, 256, launch_mpass<64, 4>, true, true},
        {"mpass K128 NT4", 128, 256, launch_mpass<128, 4>, true, true},
        {"mpass K64 NT2", 64, 256, launch_mpass<64, 2>, true, true},
        {"mpass K128 NT2", 128, 256, launch_mpass<128, 2>, true, true},
        {"piped K64 S2 U2", 64, 256, launch_piped<2, 2>, true},
        {"piped K64 S2 U1", 64, 256, launch_piped<2, 1>, true},
        {"piped K64 S2 U2 rb512", 64, 512, launch_piped<2, 2>, true},
        {"piped K96 S3 U2", 96, 256, launch_piped<3, 2>, true},
        {"piped K32 S1 U2", 32, 256, launch_piped<1, 2>, true},
        {"f4q K64 V1U2 w3 noload", 64, 256, launch_f4q<2, 3, 0>, false},
        {"f4q K64 V1U2 w3 b128", 64, 256, launch_f4q<2, 3, 2>, false},
        {"f4q K64 V1U3 w3 rb192", 64, 192, launch_f4q<3, 3>, true},
        {"f4q K64 V1U3 w3 rb384", 64, 384, launch_f4q<3, 3>, true},
        {"f4q K64 V1U4 w2", 64, 256, launch_f4q<4, 2>, true},
        {"f4q K64 V1U8 w1", 64, 256, launch_f4q<8, 1>, true},
        {"f4b K64 V1U2 w3", 64, 256, launch_f4b<3>, true},
        {"f4b K64 V1U2 w3 rb128", 64, 128, launch_f4b<3>, true},
        {"f4b K64 V1U2 w3 rb512", 64, 512, launch_f4b<3>, true},
        {"f4e K64 V1U2 w3", 64, 256, launch_f4e<3>, true},
        {"f4e K64 V1U2 w3 rb512", 64, 512, launch_f4e<3>, true},
        {"f4d K64 V1U2 asm w3", 64, 256, launch_f4d<64, 1, 2, true, 3>, true},
        {"f4d K64 V1U4 asm w3", 64, 256, launch_f4d<64, 1, 4, true, 3>, true},
        {"f4d K32 V2U2 asm w3", 32, 256, launch_f4d<32, 2, 2, true, 3>, true},
        {"f4d K16 V2U2 asm", 16, 256, launch_f4d<16, 2, 2, true>, true},
        {"f4d K16 V2U4 asm", 16, 256, launch_f4d<16, 2, 4, true>, true},
        {"f4 smem K32 V2U2", 32, 256, launch_f4<32, 2, 2, 0>, true},
        {"f4 const K32 V2U2", 32, 256, launch_f4<32, 2, 2, 1>, false},
        {"f4 copy V2U2", 32, 256, launch_f4<32, 2, 2, 2>, false},
        {"f4 readlane K32 V2U2", 32, 256, launch_f4<32, 2, 2, 3>, true},
        {"f4 smem K64 V1U4", 64, 256, launch_f4<64, 1, 4, 0>, true},
        {"f4 const K64 V1U2", 64, 256, launch_f4<64, 1, 2, 1>, false},
        {"f4 readlane K64 V1U2", 64, 256, launch_f4<64, 1, 2, 3>, true},
        {"f4 smem K16 V2U2", 16, 256, launch_f4<16, 2, 2, 0>, true},
        {"pipe K64 S2 U2 D2 rb256", 64, 256, launch_pipe<32, 2, 2, 2>, true},
        {"pipe K64 S2 U2 D3 rb256", 64, 256, launch_pipe<32, 2, 2, 3>, true},
        {"pipe K64 S2 U2 D4 rb256", 64, 256, launch_pipe<32, 2, 2, 4>, true},
        {"pipe K64 S2 U4 D2 rb256", 64, 256, launch_pipe<32, 2, 4, 2>, true},
        {"pipe K64 S2 U4 D3 rb256", 64, 256, launch_pipe<32, 2, 4, 3>, true},
        {"pipe K64 S2 U1 D4 rb256", 64, 256, launch_pipe<32, 2, 1, 4>, true},
        {"pipe K32 S2 U2 D3 rb256", 32, 256, launch_pipe<16, 2, 2, 3>, true},
        {"pipe K32 S1 U2 D3 rb256", 32, 256, launch_pipe<32, 1, 2, 3>, true},
        {"pipe K96 S3 U2 D3 rb256", 96, 256, launch_pipe<32, 3, 2, 3>, true},
        {"pipe K96 S3 U2 D4 rb256", 96, 256, launch_pipe<32, 3, 2, 4>, true},
        {"pipe K128 S4 U2 D3 rb256", 128, 256, launch_pipe<32, 4, 2, 3>, true},
    };
    for (auto& v : vs)
        if (v.exact && !(only && !strcmp(only, "copy")) && (!only || strstr(v.name, only))) printf("check %-28s %s\n", v.name, check(v) ? "bit-exact" : "FAILED");
    Lab L;
    L.rows = rows;
    L.width = (ncols + 15) / 16 * 16;
    L.ld = L.width >= 4096 ? (L.width + 511) / 512 * 512 : L.width;
    if (getenv("LAB_LD")) L.ld = atoll(getenv("LAB_LD"));
    printf("tableau %ld x %ld (width %ld, ld %ld): %.2f GB\n", (long)rows, (long)ncols, (long)L.width, (long)L.ld,
           rows * L.ld * 8 / 1e9);
    CK(hipMalloc(&L.T, rows * L.ld * 8));
    L.To = L.T;   // in place, as the product's pass without lookahead
    if (getenv("LAB_OOP")) {   // out of place, as the product's pass under lookahead
        CK(hipMalloc(&L.To, rows * L.ld * 8));
        CK(hipMemset(L.To, 0, rows * L.ld * 8));
        printf("out of place\n");
    }
    CK(hipMalloc(&L.Cr, rows * 128 * 8));
    CK(hipMalloc(&L.P, (int64_t)128 * L.ld * 8));
    fill_kernel<<<4096, 256>>>(L.T, rows * L.ld, 1);
    fill_kernel<<<1024, 256>>>(L.Cr, rows * 128, 2);
    fill_kernel<<<1024, 256>>>(L.P, (int64_t)128 * L.ld, 3);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 16.0 * rows * ncols;




    if (only && !strcmp(only, "lat")) {
        double* out;
        CK(hipMalloc(&out, 256 * 8192 * 8));
        const int iters = 2048;
        for (int mode = 1; mode <= 2; ++mode)
            for (int nch : {1, 2, 4, 8})
                for (int w : {1, 2, 3, 4}) {
                    const int wg = 256 * w;   // w waves per SIMD
                    auto go = [&]() {
#define LK(M, N) lat_kernel<M, N><<<wg, 256>>>(out, 0.5, iters)
                        if (mode == 1) { if (nch == 1) LK(1, 1); else if (nch == 2) LK(1, 2); else if (nch == 4) LK(1, 4); else LK(1, 8); }
                        else { if (nch == 1) LK(2, 1); else if (nch == 2) LK(2, 2); else if (nch == 4) LK(2, 4); else LK(2, 8); }
#undef LK
                    };
                    go();
                    CK(hipDeviceSynchronize());
                    CK(hipEventRecord(e0, 0));
                    go();
                    CK(hipEventRecord(e1, 0));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    const double fl = 2.0 * 8.0 * nch * iters * wg * 256;
                    printf("lat %s chains %d waves/SIMD %d: %.1f TF/s\n", mode == 1 ? "fmac_dpp" : "fma     ", nch, w,
                           fl / ms / 1e9);
                }
        return 0;
    }
    if (only && !strcmp(only, "valu")) {
        double* out;
        CK(hipMalloc(&out, 256 * 8192 * 8));
        const int iters = 4096;
        for (int mode = 0; mode < 3; ++mode)
            for (int wg : {1024, 2048, 4096}) {
                auto go = [&]() {
                    if (mode == 0) valu_kernel<0><<<wg, 256>>>(out, 0.5, iters);
                    else if (mode == 1) valu_kernel<1><<<wg, 256>>>(out, 0.5, iters);
                    else valu_kernel<2><<<wg, 256>>>(out, 0.5, iters);
                };
                go();
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(e0, 0));
                go();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                const double fl = 2.0 * 64.0 * iters * wg * 256;
                printf("valu mode %d wgs %d: %.3f ms  %.1f TF/s\n", mode, wg, ms, fl / ms / 1e9);
            }
        return 0;
    }
    if (only && !strcmp(only, "hetero")) {
        // round 5: the VALU (DPP, f4r) and the matrix-core (mpass4) passes side by side on every CU,
        // each on a share of the columns, as two concurrent launches whose occupancy is held by
        // dynamic LDS (f4r nw WGs per CU, mpass4 nm per CU): both pipes busy at once
        hipStream_t sa, sb;
        CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
        hipEvent_t a0, a1, b1;
        CK(hipEventCreate(&a0));
        CK(hipEventCreate(&a1));
        CK(hipEventCreate(&b1));
        const int rb = 768;
        struct H { double frac; int nw, nm; };
        for (const H h : {H{0.0, 0, 3}, H{1.0, 3, 0}, H{0.25, 1, 2}, H{0.33, 1, 2}, H{0.4, 1, 2}, H{0.5, 1, 2},
                          H{0.33, 1, 3}, H{0.5, 2, 1}})
        for (int rep2 = 0; rep2 < 1; ++rep2) {
            const int64_t wa = (int64_t)(L.width * h.frac / 256.0 + 0.5) * 256;   // f4r's columns
            Lab La = L, Lb = L;
            La.width = wa;
            Lb.T = L.T + wa;
            Lb.To = L.To + wa;
            Lb.P = L.P + wa;
            Lb.width = L.width - wa;
            // mpass4 WG = 18 KiB static + 2 KiB dynamic = 20 KiB; f4r takes the rest, nw per CU
            const size_t dynb = (h.nm && h.nw) ? 2048 : 0;
            const size_t dyna = h.nw ? (size_t)(163840 - h.nm * 20480 - 1024) / h.nw : 0;
            auto go = [&]() {
                if (wa > 0) {
                    dim3 grid((unsigned)((La.width + 255) / 256), (unsigned)((La.rows + rb - 1) / rb));
                    f4r_kernel<true, 4, 3, 3><<<grid, 256, std::max(dyna, (size_t)4 * 3 * 1024 * 4), sa>>>(
                        La.T, La.To, La.ld, La.rows, La.width, La.Cr, La.P, rb);
                }
                if (Lb.width > 0) {
                    dim3 grid((unsigned)((Lb.width + 127) / 128), (unsigned)((Lb.rows + rb - 1) / rb));
                    mpass4_kernel<64, 2, 3><<<grid, 256, dynb, sb>>>(Lb.T, Lb.To, Lb.ld, Lb.rows, Lb.width, Lb.Cr,
                                                                     Lb.P, rb);
                }
            };
            go();
            CK(hipDeviceSynchronize());
            std::vector<float> ms(reps);
            for (int r = 0; r < reps; ++r) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(a0, 0));
                CK(hipStreamWaitEvent(sa, a0, 0));
                CK(hipStreamWaitEvent(sb, a0, 0));
                go();
                CK(hipEventRecord(a1, sa));
                CK(hipEventRecord(b1, sb));
                CK(hipStreamWaitEvent(0, a1, 0));
                CK(hipStreamWaitEvent(0, b1, 0));
                hipEvent_t e2;
                CK(hipEventCreate(&e2));
                CK(hipEventRecord(e2, 0));
                CK(hipEventSynchronize(e2));
                CK(hipEventElapsedTime(&ms[r], a0, e2));
                CK(hipEventDestroy(e2));
            }
            std::sort(ms.begin(), ms.end());
            printf("hetero f4r share %.2f (%ld cols, %d WG/CU, dyn %zu) + mpass4 (%d WG/CU, dyn %zu): median %.3f ms  %6.0f GB/s\n",
                   h.frac, (long)wa, h.nw, dyna, h.nm, dynb, ms[reps / 2], bytes / ms[reps / 2] / 1e6);
            fflush(stdout);
        }
        return 0;
    }
    if (only && !strcmp(only, "copyw")) {
        struct C { int nth, rb; };
        std::vector<C> cs;
        for (int rb : {8, 32, 256, 768})
            for (int nth : {256, 512, 768, 1024}) cs.push_back({nth, rb});
        for (int rep2 = 0; rep2 < 2; ++rep2)
        for (auto& c : cs) {
            auto go = [&]() {
                dim3 grid((unsigned)((L.width + c.nth - 1) / c.nth), (unsigned)((L.rows + c.rb - 1) / c.rb));
                switch (c.nth) {
                    case 256: copyw_kernel<256><<<grid, 256>>>(L.T, L.To, L.ld, L.rows, L.width, c.rb); break;
                    case 512: copyw_kernel<512><<<grid, 512>>>(L.T, L.To, L.ld, L.rows, L.width, c.rb); break;
                    case 768: copyw_kernel<768><<<grid, 768>>>(L.T, L.To, L.ld, L.rows, L.width, c.rb); break;
                    default: copyw_kernel<1024><<<grid, 1024>>>(L.T, L.To, L.ld, L.rows, L.width, c.rb); break;
                }
            };
            go();
            CK(hipDeviceSynchronize());
            std::vector<float> ms(reps);
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e0, 0));
                go();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms[r], e0, e1));
            }
            std::sort(ms.begin(), ms.end());
            printf("copyw nth=%4d rb=%4d  median %.3f ms  %6.0f GB/s\n", c.nth, c.rb, ms[reps / 2],
                   bytes / ms[reps / 2] / 1e6);
            fflush(stdout);
        }
        return 0;
    }
    if (only && !strcmp(only, "copyp")) {
        struct C { int U, rb, occ, G, tf; };
        std::vector<C> cs;
        for (int U : {1, 2})
            for (int rb : {8, 16})
                for (int G : {2, 3, 4, 8})
                    for (int tf : {1, 0}) cs.push_back({U, rb, U == 1 ? 4 : 2, G, tf});
        cs.push_back({2, 8, 2, 0, 1});   // G = 0: plain short bands (reference)
        const int ntile = (int)((L.width + 511) / 512);
        for (auto& c : cs) {
            const size_t dyn = c.occ ? (size_t)160 * 1024 / c.occ - 512 : 0;
            auto go = [&]() {
                if (c.G == 0) {
                    dim3 grid((unsigned)ntile, (unsigned)((L.rows + c.rb - 1) / c.rb));
                    copy_kernel<2><<<grid, 256, dyn>>>(L.T, L.ld, L.rows, L.width, c.rb);
                    return;
                }
                const unsigned nb = (unsigned)(ntile * c.G);
                if (c.U == 1) copyp_kernel<1><<<nb, 256, dyn>>>(L.T, L.ld, L.rows, L.width, c.rb, c.G, c.tf);
                else copyp_kernel<2><<<nb, 256, dyn>>>(L.T, L.ld, L.rows, L.width, c.rb, c.G, c.tf);
            };
            go();
            CK(hipDeviceSynchronize());
            std::vector<float> ms(reps);
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e0, 0));
                go();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms[r], e0, e1));
            }
            std::sort(ms.begin(), ms.end());
            printf("copyp U=%d rb=%3d occ=%d G=%d tf=%d  median %.3f ms  %6.0f GB/s\n", c.U, c.rb, c.occ, c.G, c.tf,
                   ms[reps / 2], bytes / ms[reps / 2] / 1e6);
            fflush(stdout);
        }
        return 0;
    }
    if (only && !strcmp(only, "copy")) {
        struct C { int U, rb, occ; };
        std::vector<C> cs;
        for (int U : {1, 2, 4, 8})
            for (int rb : {8, 32, 256})
                for (int occ : {0, 4, 2})
                    if (rb % U == 0) cs.push_back({U, rb, occ});
        for (auto& c : cs) {
            const size_t dyn = c.occ ? (size_t)160 * 1024 / c.occ - 512 : 0;
            auto go = [&]() {
                dim3 grid((unsigned)((L.width + 511) / 512), (unsigned)((L.rows + c.rb - 1) / c.rb));
                switch (c.U) {
                    case 1: copy_kernel<1><<<grid, 256, dyn>>>(L.T, L.ld, L.rows, L.width, c.rb); break;
                    case 2: copy_kernel<2><<<grid, 256, dyn>>>(L.T, L.ld, L.rows, L.width, c.rb); break;
                    case 4: copy_kernel<4><<<grid, 256, dyn>>>(L.T, L.ld, L.rows, L.width, c.rb); break;
                    default: copy_kernel<8><<<grid, 256, dyn>>>(L.T, L.ld, L.rows, L.width, c.rb); break;
                }
            };
            go();
            CK(hipDeviceSynchronize());
            std::vector<float> ms(reps);
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e0, 0));
                go();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                CK(hipEventElapsedTime(&ms[r], e0, e1));
            }
            std::sort(ms.begin(), ms.end());
            printf("copy U=%d rb=%4d occ=%d  median %.3f ms  %6.0f GB/s\n", c.U, c.rb, c.occ, ms[reps / 2],
                   bytes / ms[reps / 2] / 1e6);
            fflush(stdout);
        }
        return 0;
    }
    for (auto& v : vs) {
        if (only && !strstr(v.name, only)) continue;
        v.fn(L, v.K, v.rb, 0);   // warm
        CK(hipDeviceSynchronize());
        std::vector<float> ms(reps);
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, 0));
            v.fn(L, v.K, v.rb, 0);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms[r], e0, e1));
        }
        std::vector<float> s = ms;
        std::sort(s.begin(), s.end());
        const float med = s[reps / 2];
        printf("%-28s K=%2d rb=%4d  median %.3f ms  %6.0f GB/s  %.4f ms/step\n", v.name, v.K, v.rb, med,
               bytes / med / 1e6, med / v.K);
        fflush(stdout);
    }
    return 0;
}
