// dlp_cluster.hip — small LPs (a tableau that fits the LDS of the chip's CUs):
// the whole solve window in ONE launch, the tableau resident in LDS, spread
// over G workgroups (one per CU) by column slices.  For such tableaus the
// multi-kernel pivot is launch- and latency-bound (C1 200 x 400: ~16 us per
// pivot in 3 launches, C4 256 x 512: ~14 us), while the arithmetic is a few
// hundred KB of LDS traffic per pivot.
//
// Per pivot, every workgroup (the exact rule of
// dlp.h, bit-identical to the eager kernels and the oracle):
//   1. prices its columns of the objective row (LDS), publishes the partial
//      and its local choice's column; all read the G partials and reduce
//      them in the same order -> the same q everywhere;
//   2. takes column q from its owner's published copy;
//   3. runs the whole ratio test itself (redundantly: colq, its copy of the
//      RHS column and of the basis, all in LDS) -> the same p everywhere;
//   4. normalises its part of row p (IEEE division) and eliminates its slice;
//      advances its RHS copy with the same fma.
// One hand-off per pivot: each workgroup publishes its pricing partial and,
// speculatively, the column of its own local choice as data-tagged granules
// (gput / gget); every workgroup polls the G partials, and then the winner's
// column, which was published in the same burst.
// Every wait is bounded: a stall ends the window with DLP_ERR_HIP in the
// state, never a hang.  All G workgroups must be resident at once: the
// launcher keeps G <= the CU count with one workgroup's LDS > half a CU's.
//
// Reference analogs as for the other pivot kernels: first-wins scans
// R/global_problem.cpp:335-361 (pricing), the tight-set test :372-380
// (ratio), the 2x2 basis solve :393-405 (elimination).
#include <hip/hip_runtime.h>

#include "dlp_internal.h"

namespace dlp {
namespace {

#include "dlp_device.h"

typedef unsigned int u4v __attribute__((ext_vector_type(4)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
constexpr int kSpin = 1 << 24;    // bounded waits (each poll sleeps ~64 cycles)

// One workgroup's LDS image (dynamic): slice T[(m+1)][cw] (row-major, stride
// cw), colq[m+1], rhs[m] (copy of the RHS column), prow[cw], basis[m].
struct ClusterArgs {
    double* T;            // HBM tableau (rows m+1, stride ld): loaded at the start, stored at the end
    int64_t ld;
    int m, n, N;          // N = n + m; column N = RHS
    int cw;               // columns per workgroup
    int64_t max_pivots;   // pivots this window
    int pricing;
    double tol_dj, tol_piv;
    DevState* st;
    int32_t* basis;       // global basis (m)
    dlp_pivot* log;
    int64_t log_cap;
    uint64_t* gran;       // [2][G][gstride] granules: partial (4), then colq (2 per row)
    uint64_t* stamps;     // diagnostic build only (DLP_CLUSTER_STAMPS): s_memtime per phase
    int64_t gstride;      // granules per workgroup slot: 4 + 2 (m + 1), rounded to 16
};

// Data-tagged granules: one 8-byte write-through store carries a 32-bit payload
// and the pivot's tag; a reader polls the word itself until the tag matches, so
// no flag, counter, drain or fence orders anything (MI355X_MICROARCH.md,
// handoff-1to1: 8-byte {data, tag} granules written by ONE sc1 store).
__device__ inline void gput(uint64_t* p, uint32_t tag, uint32_t v) {
    __hip_atomic_store(p, ((uint64_t)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// NG granules at p[0], p[stride], ...: every load of a round is issued before
// any tag is checked, so a round costs one memory round trip, not NG.
template <int NG>
__device__ inline bool gget(const uint64_t* p, int stride, uint32_t tag, uint32_t (&v)[NG]) {
    for (int it = 0; it < kSpin; ++it) {
        uint64_t x[NG];
#pragma unroll
        for (int e = 0; e < NG; ++e)
            x[e] = __hip_atomic_load(p + e * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool all = true;
#pragma unroll
        for (int e = 0; e < NG; ++e) all = all && (uint32_t)(x[e] >> 32) == tag;
        if (all) {
#pragma unroll
            for (int e = 0; e < NG; ++e) v[e] = (uint32_t)x[e];
            return true;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return false;
}

__global__ __launch_bounds__(256) void cluster_solve_kernel(ClusterArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    __shared__ PricePart lds_pp[4];
    __shared__ Cand lds_c[4];
    __shared__ int s_flag;
    const int G = gridDim.x, g = blockIdx.x, tid = threadIdx.x;
    const int m = a.m, N = a.N, cw = a.cw, W = N + 1;
    const int c0 = g * cw, c1 = min(c0 + cw, W), nc = max(c1 - c0, 0);
    double* T = smem;                               // (m+1) x cw
    double* colq = T + (size_t)(m + 1) * cw;        // m+1
    double* rhs = colq + (m + 1);                   // m
    double* prow = rhs + m;                         // cw
    int32_t* basis = (int32_t*)(prow + cw);         // m

    DevState* st = a.st;
    const int status0 = st->status;
    if (status0 != DLP_RUNNING) return;
    int bland = st->bland;
    int64_t np = st->npivots;

    // load the slice, the RHS copy and the basis copy
    for (int e = tid; e < (m + 1) * cw; e += blockDim.x) {
        const int i = e / cw, jl = e - i * cw;
        T[e] = jl < nc ? a.T[(int64_t)i * a.ld + c0 + jl] : 0.0;
    }
    for (int i = tid; i < m; i += blockDim.x) {
        rhs[i] = a.T[(int64_t)i * a.ld + N];
        basis[i] = a.basis[i];
    }
    __syncthreads();

    if (tid == 0) s_flag = 1;
    __syncthreads();
    int status = DLP_RUNNING;
    int64_t k = 0;
    for (; k < a.max_pivots; ++k) {
        const int par = (int)(k & 1);
        if (a.stamps && tid == 0 && k < 64) a.stamps[((size_t)g * 64 + k) * 16 + 0] = __builtin_amdgcn_s_memtime();
        // ---- 1. this slice's pricing partial and the column of its local choice,
        //         published as data-tagged granules (tag = k + 1 in the high word)
        PricePart acc = pp_empty();
        for (int jl = tid; jl < nc; jl += blockDim.x) {
            const int j = c0 + jl;
            if (j < N) {
                const double z = T[(size_t)m * cw + jl];
                if (z < acc.zmin) { acc.zmin = z; acc.jmin = j; }
                if (z < -a.tol_dj && acc.jbland == kNoIndex) acc.jbland = j;
            }
        }
        acc = block_price(acc, lds_pp);
        const uint32_t tag = (uint32_t)(k + 1);
        uint64_t* mine = a.gran + ((size_t)par * G + g) * a.gstride;
        {
            const int ql = bland ? acc.jbland
                                 : ((acc.jmin != kNoIndex && acc.zmin < -a.tol_dj) ? acc.jmin : kNoIndex);
            if (tid < 4) {
                const uint64_t zb = __builtin_bit_cast(uint64_t, acc.zmin);
                const uint32_t w = tid == 0 ? (uint32_t)zb : tid == 1 ? (uint32_t)(zb >> 32)
                                 : tid == 2 ? (uint32_t)acc.jmin : (uint32_t)acc.jbland;
                gput(mine + tid, tag, w);
            }
            if (ql != kNoIndex)   // speculative: this slice's choice may be the global one
                for (int i = tid; i <= m; i += blockDim.x) {
                    const uint64_t v = __builtin_bit_cast(uint64_t, T[(size_t)i * cw + (ql - c0)]);
                    gput(mine + 4 + 2 * i, tag, (uint32_t)v);
                    gput(mine + 5 + 2 * i, tag, (uint32_t)(v >> 32));
                }
        }
        if (a.stamps && tid == 0 && k < 64) a.stamps[((size_t)g * 64 + k) * 16 + 1] = __builtin_amdgcn_s_memtime();
        // every workgroup's partial (granule polls, bounded), the same reduction order
        bool ok = true;
        PricePart tot = pp_empty();
        for (int w = tid; w < G; w += blockDim.x) {
            const uint64_t* gw = a.gran + ((size_t)par * G + w) * a.gstride;
            uint32_t v[4];
            ok = gget<4>(gw, 1, tag, v) && ok;
            PricePart o;
            o.zmin = __builtin_bit_cast(double, (uint64_t)v[0] | ((uint64_t)v[1] << 32));
            o.jmin = (int32_t)v[2];
            o.jbland = (int32_t)v[3];
            pp_combine(tot, o);
        }
        if (!ok) s_flag = 0;
        tot = block_price(tot, lds_pp);
        if (s_flag == 0) { status = DLP_ERR_HIP; break; }
        int q;
        if (bland)
            q = tot.jbland;
        else
            q = (tot.jmin != kNoIndex && tot.zmin < -a.tol_dj) ? tot.jmin : kNoIndex;
        if (q == kNoIndex) { status = DLP_OK; break; }

        if (a.stamps && tid == 0 && k < 64) a.stamps[((size_t)g * 64 + k) * 16 + 2] = __builtin_amdgcn_s_memtime();
        // ---- 2. column q: the owner's published copy (its local choice was q)
        const int owner = q / cw;
        if (g == owner) {
            for (int i = tid; i <= m; i += blockDim.x) colq[i] = T[(size_t)i * cw + (q - c0)];
        } else {
            const uint64_t* go = a.gran + ((size_t)par * G + owner) * a.gstride;
            // rows tid, tid + 256, ... in rounds of four rows (8 granules, loads issued
            // together); rows past m re-read row m's granules
            for (int i0 = tid; i0 <= m; i0 += 4 * (int)blockDim.x) {
                int rr[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) rr[r] = min(i0 + r * (int)blockDim.x, m);
                bool got = false;
                for (int it = 0; it < kSpin && !got; ++it) {
                    uint64_t x[8];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        x[2 * r] = __hip_atomic_load(go + 4 + 2 * rr[r], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                        x[2 * r + 1] = __hip_atomic_load(go + 5 + 2 * rr[r], __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                    }
                    bool all = true;
#pragma unroll
                    for (int e = 0; e < 8; ++e) all = all && (uint32_t)(x[e] >> 32) == tag;
                    if (all) {
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            colq[rr[r]] = __builtin_bit_cast(
                                double, (uint64_t)(uint32_t)x[2 * r] | ((uint64_t)(uint32_t)x[2 * r + 1] << 32));
                        got = true;
                    } else {
                        __builtin_amdgcn_s_sleep(1);
                    }
                }
                ok = ok && got;
            }
            if (!ok) s_flag = 0;
        }
        __syncthreads();
        if (s_flag == 0) { status = DLP_ERR_HIP; break; }

        if (a.stamps && tid == 0 && k < 64) a.stamps[((size_t)g * 64 + k) * 16 + 3] = __builtin_amdgcn_s_memtime();
        // ---- 3. ratio test over every row (the same answer in every workgroup)
        Cand best = cand_empty();
        for (int i = tid; i < m; i += blockDim.x) {
            const double av = colq[i];
            if (av > a.tol_piv) {
                double b = rhs[i];
                if (!(b > 0.0)) b = 0.0;
                Cand c;
                c.ratio = b / av;
                c.basis_var = basis[i];
                c.row = i;
                c.valid = 1;
                c.pad0 = 0;
                c.pivot = av;
                if (cand_better(c, best)) best = c;
            }
        }
        if (a.stamps && tid == 0 && k < 64) a.stamps[((size_t)g * 64 + k) * 16 + 6] = __builtin_amdgcn_s_memtime();
        best = block_cand(best, lds_c);
        if (!best.valid) { status = DLP_UNBOUNDED; break; }
        const int p = best.row;
        const double piv = best.pivot;
        const int leaving = basis[p];
        bland = (a.pricing == DLP_PRICING_BLAND) ? 1 : (best.ratio == 0.0 ? 1 : 0);
        if (g == 0 && tid == 0 && a.log && np < a.log_cap) {
            dlp_pivot* e = a.log + np;
            e->q = q;
            e->p = p;
            e->leaving = leaving;
            e->pad = 0;
            e->ratio = best.ratio;
        }

        if (a.stamps && tid == 0 && k < 64) a.stamps[((size_t)g * 64 + k) * 16 + 4] = __builtin_amdgcn_s_memtime();
        // ---- 4. pivot row (IEEE division) and elimination of this slice
        for (int jl = tid; jl < nc; jl += blockDim.x) prow[jl] = T[(size_t)p * cw + jl] / piv;
        const double prN = rhs[p] / piv;   // = the RHS owner's prow at column N
        if (a.stamps && tid == 0 && k < 64) a.stamps[((size_t)g * 64 + k) * 16 + 7] = __builtin_amdgcn_s_memtime();
        __syncthreads();
        if (tid == 0) basis[p] = q;
        // thread -> (column tj, first row ti), rows strided by rpi: no division per element
        for (int jb = 0; jb < nc; jb += blockDim.x) {
            const int span = min((int)blockDim.x, nc - jb);
            const int rpi = blockDim.x / span, tj = tid % span, ti = tid / span;
            if (ti < rpi) {
                const int jl = jb + tj;
                const double pj = prow[jl];
                // 8 rows per round: all LDS loads issued, then selects (an untouched element
                // is stored back unchanged), then the stores
                for (int i0 = ti; i0 <= m; i0 += 8 * rpi) {
                    double t[8], f[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int i = min(i0 + u * rpi, m);
                        f[u] = colq[i];
                        t[u] = T[(size_t)i * cw + jl];
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int i = i0 + u * rpi;
                        const double v = __builtin_fma(-f[u], pj, t[u]);
                        const double nv = (i == p) ? pj : (f[u] != 0.0 ? v : t[u]);
                        if (i <= m) T[(size_t)i * cw + jl] = nv;
                    }
                }
            }
        }
        if (a.stamps && tid == 0 && k < 64) a.stamps[((size_t)g * 64 + k) * 16 + 8] = __builtin_amdgcn_s_memtime();
        for (int i = tid; i < m; i += blockDim.x) {
            if (i == p) {
                rhs[i] = prN;
            } else {
                const double f = colq[i];
                if (f != 0.0) rhs[i] = __builtin_fma(-f, prN, rhs[i]);
            }
        }
        __syncthreads();
        if (N >= c0 && N < c1 && tid == 0 && a.log && np < a.log_cap)
            a.log[np].objective = T[(size_t)m * cw + (N - c0)];
        if (a.stamps && tid == 0 && k < 64) a.stamps[((size_t)g * 64 + k) * 16 + 5] = __builtin_amdgcn_s_memtime();
        ++np;
    }

    // store the slice back; workgroup 0 publishes the state and the basis
    for (int e = tid; e < (m + 1) * cw; e += blockDim.x) {
        const int i = e / cw, jl = e - i * cw;
        if (jl < nc) a.T[(int64_t)i * a.ld + c0 + jl] = T[e];
    }
    if (g == 0) {
        for (int i = tid; i < m; i += blockDim.x) a.basis[i] = basis[i];
        if (tid == 0) {
            st->npivots = np;
            st->bland = bland;
            if (status != DLP_RUNNING) st->status = status;
        }
    } else if (status == DLP_ERR_HIP && tid == 0) {
        st->status = DLP_ERR_HIP;
    }
}

}  // namespace

int64_t cluster_gstride(int64_t m) { return (4 + 2 * (m + 1) + 15) / 16 * 16; }

size_t cluster_lds_bytes(int64_t m, int cw) {
    return sizeof(double) * ((size_t)(m + 1) * cw + (m + 1) + m + cw) + sizeof(int32_t) * m + 16;
}

// Workgroups for an (m+1) x (N+1) tableau: the fewest whose slices stay within
// 64 KiB of LDS (the balance of elimination bandwidth against the fan-in of the
// two waits), else the fewest that fit at all; every workgroup keeps >= 1
// column; 0 when even max_wg workgroups would not hold the tableau.
int cluster_plan(int64_t m, int64_t N, int max_wg, int* cw_out) {
    const int64_t W = N + 1;
    const size_t cap = 160 * 1024 - 1024;   // the kernel's static LDS + margin
    const size_t target = 64 * 1024;
    for (const size_t lim : {target, cap}) {
        for (int G = 1; G <= max_wg && G <= W; ++G) {
            const int cw = (int)((W + G - 1) / G);
            if ((int64_t)(G - 1) * cw >= W) continue;   // a workgroup without columns
            if (cluster_lds_bytes(m, cw) <= lim) {
                if (cw_out) *cw_out = cw;
                return G;
            }
        }
    }
    return 0;
}

int64_t cluster_granules(int64_t m, int nwg) { return 2 * (int64_t)nwg * cluster_gstride(m); }

hipError_t launch_cluster(const Geometry& g, int64_t m, int64_t n, int nwg, int cw, DevState* st,
                          int32_t* basis, dlp_pivot* log, int64_t log_cap, uint64_t* gran,
                          int64_t max_pivots, int pricing, double tol_dj, double tol_piv,
                          hipStream_t s, uint64_t* stamps) {
    ClusterArgs a;
    a.T = g.T;
    a.ld = g.ld;
    a.m = (int)m;
    a.n = (int)n;
    a.N = (int)(n + m);
    a.cw = cw;
    a.max_pivots = max_pivots;
    a.pricing = pricing;
    a.tol_dj = tol_dj;
    a.tol_piv = tol_piv;
    a.st = st;
    a.basis = basis;
    a.log = log;
    a.log_cap = log_cap;
    a.gran = gran;
    a.stamps = stamps;
    a.gstride = cluster_gstride(m);
    const size_t lds = cluster_lds_bytes(m, cw);
    hipError_t e = hipFuncSetAttribute((const void*)cluster_solve_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(gran, 0, sizeof(uint64_t) * cluster_granules(m, nwg), s);   // tags restart at 1
    if (e != hipSuccess) return e;
    cluster_solve_kernel<<<nwg, 256, lds, s>>>(a);
    return hipGetLastError();
}

}  // namespace dlp
