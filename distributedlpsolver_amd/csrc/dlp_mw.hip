// dlp_mw.hip — SURVEY.md §8f row f3: the reference's multiplicative-weights
// (MW) iteration, sort mode, on the GPU.  One MW iteration =
//   weighted budget B = sum_fixed(w_a B_a)                 R/allocation_mw.cpp:102-108
//   per impression: upper envelope of (price*w, price) + origin, envelope
//     points (u, v) and budget cutoffs                      R/subproblem.cpp:186-233,
//                                                           R/upper_envelope.cpp:15-38
//   global split of B over envelope regions by slope       R/global_problem.cpp:224-255
//   per impression: primal x from the allocated region     R/global_problem.cpp:325-412
//   dual value = sum over impressions of u*beta + v        R/global_problem.cpp:306-322
//   running average of x                                   R/instance.cpp:143-152
//   per advertiser: slack, average slack, weight update    R/allocation_mw.cpp:163-203
// with the fp64 spec of DESIGN.md §9 (fixed tie orders, fixed-order sums,
// deterministic exp), so the result is bit-identical to the CPU restatement.
//
// Layout: bids in impression-major CSR (advertiser ascending inside an
// impression) for the envelope/primal kernels, plus an advertiser-major index
// for the slack gather (no float atomics: every sum has a fixed order).
// Kernels: one wave per impression for the envelope (bitonic sort of the
// points in LDS, then the monotone chain on one lane); a stable hipCUB radix
// sort of all regions by slope; a chunked budget prefix; one lane per
// impression / advertiser for primal and weights.
//
// Binary (threshold-search) mode, R/global_problem.cpp:46-222, 283-292, the
// mode R/main.cpp:36 runs (spec: oracle/oracle_mw.cpp header): no sort.  The
// search state lives on the device; one launch per search level evaluates the
// nr critical ratios over all regions (one lane per impression, a 256-lane
// tree per block) and the block that finishes last reduces the block sums
// and applies the reference's bracket / expand / stop rule, so levels queue
// back to back with no host round trip (the host polls `done` once per batch
// of launches).  Instances whose impressions fit one workgroup run the whole
// search inside one launch.  The tie allocation is the one serial step of the
// reference (remaining budget shrinks tie by tie): compacted tie list, one
// wave walking it with the budget in a uniform register.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "dlp_host.h"
#include "dlp_internal.h"

namespace dlp {
namespace mw {

constexpr int kDegMax = 1024;   // points per impression (bids + origin) the envelope kernel holds
constexpr int kChunk = 256;     // budget-prefix chunk (spec)
constexpr double kHullTol = 1e-14;   // R/subproblem.cpp:205, 224

// Deterministic exp (spec): x = k ln2 + r with k = rint(x / ln2), r by two
// fma with ln2 split hi/lo, e^r by the degree-13 Taylor polynomial in Horner
// form with fma, scaled by 2^k.  Identical IEEE operation sequence on host
// oracle and device, hence bit-identical weights.
__device__ inline double dexp(double x) {
    const double inv_ln2 = 0x1.71547652b82fep+0;
    const double ln2_hi = 0x1.62e42fefa39efp-1;
    const double ln2_lo = 0x1.abc9e3b39803fp-56;
    const double k = __builtin_rint(x * inv_ln2);
    double r = __builtin_fma(-k, ln2_hi, x);
    r = __builtin_fma(-k, ln2_lo, r);
    double p = 0x1.6124613a86d09p-33;              // 1/13!
    p = __builtin_fma(p, r, 0x1.1eed8eff8d898p-29);  // 1/12!
    p = __builtin_fma(p, r, 0x1.ae64567f544e4p-26);  // 1/11!
    p = __builtin_fma(p, r, 0x1.27e4fb7789f5cp-22);  // 1/10!
    p = __builtin_fma(p, r, 0x1.71de3a556c734p-19);  // 1/9!
    p = __builtin_fma(p, r, 0x1.a01a01a01a01ap-16);  // 1/8!
    p = __builtin_fma(p, r, 0x1.a01a01a01a01ap-13);  // 1/7!
    p = __builtin_fma(p, r, 0x1.6c16c16c16c17p-10);  // 1/6!
    p = __builtin_fma(p, r, 0x1.1111111111111p-7);   // 1/5!
    p = __builtin_fma(p, r, 0x1.5555555555555p-5);   // 1/4!
    p = __builtin_fma(p, r, 0x1.5555555555555p-3);   // 1/3!
    p = __builtin_fma(p, r, 0.5);
    p = __builtin_fma(p, r, 1.0);
    p = __builtin_fma(p, r, 1.0);
    return __builtin_ldexp(p, (int)k);
}

// One lane's chain of the fixed-order sum: x[lane], x[lane+64], ... added in
// order; loads issued 16 ahead of the dependent adds (same order, no stall per
// element).
__device__ inline double lane_chain(const double* __restrict__ x, int64_t n, int lane) {
    constexpr int U = 16;
    double acc = 0.0;
    int64_t k = lane;
    for (; k + 64 * (U - 1) < n; k += 64 * U) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = x[k + 64 * u];
#pragma unroll
        for (int u = 0; u < U; ++u) acc = acc + v[u];
    }
    for (; k < n; k += 64) acc = acc + x[k];
    return acc;
}

// sum_fixed by one wave (spec: 64 strided sequential chains, halving tree).
__device__ inline double wave_sum_fixed(const double* x, int64_t n, int lane) {
    double a = lane_chain(x, n, lane);
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) a = a + __shfl_down(a, w);
    return a;
}

// Fixed-order sum (spec): 64 strided sequential chains, then the halving tree.
__global__ __launch_bounds__(64) void sum_fixed_kernel(const double* __restrict__ x, int64_t n,
                                                       double* __restrict__ out) {
    const double acc = wave_sum_fixed(x, n, threadIdx.x);
    if (threadIdx.x == 0) *out = acc;
}

__global__ void weighted_budget_kernel(const double* __restrict__ w, const double* __restrict__ b,
                                       int A, double* __restrict__ wb) {
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a < A) wb[a] = w[a] * b[a];
}

struct HullPt {
    double c, p;
    int adv;
};

__device__ inline bool hull_before(const HullPt& a, const HullPt& b) {   // (c desc, p desc, adv asc)
    if (a.c != b.c) return a.c > b.c;
    if (a.p != b.p) return a.p > b.p;
    return a.adv < b.adv;
}

// Monotone chain over the n sorted points (lane 0), envelope points and
// cutoffs to the impression's slots (R/upper_envelope.cpp:15-38,
// R/subproblem.cpp:186-233).
__device__ inline void envelope_chain(const double* sc, const double* sp, const int* sa, int* stk, int n,
                                      int64_t b0, int i, double* env_u, double* env_v, double* cut,
                                      int32_t* hull_h) {
    (void)sa;
    int h = 0;
    for (int q = 0; q < n; ++q) {
        while (h >= 2) {
            const int O = stk[h - 2], Aq = stk[h - 1];
            const double d1 = (sc[Aq] - sc[O]) * (sp[q] - sp[O]);
            const double d2 = (sp[Aq] - sp[O]) * (sc[q] - sc[O]);
            if (d1 - d2 <= kHullTol) --h; else break;
        }
        stk[h++] = q;
    }
    const int64_t bu = b0 + i, bc = b0 + 2 * (int64_t)i;
    {
        const int q = stk[h - 2];
        env_u[bu] = sp[q] / sc[q];
        env_v[bu] = 0.0;
    }
    int e = 1;
    for (int k = h - 2; k > 0; --k, ++e) {
        const int q1 = stk[k - 1], q0 = stk[k];
        const double uu = (sp[q1] - sp[q0]) / (sc[q1] - sc[q0]);
        env_u[bu + e] = uu;
        const double t = sc[q1] * uu;
        env_v[bu + e] = sp[q1] - t;
    }
    env_u[bu + e] = 0.0;
    env_v[bu + e] = sp[stk[0]];
    cut[bc] = 0.0;
    for (int k = 0; k < h - 1; ++k) {
        const double du = env_u[bu + k] - env_u[bu + k + 1];
        cut[bc + k + 1] = (du > kHullTol) ? (env_v[bu + k + 1] - env_v[bu + k]) / du : cut[bc + k];
    }
    cut[bc + h] = DBL_MAX;
    hull_h[i] = h;
}

// One 64-lane workgroup per impression: points to LDS, bitonic sort, monotone
// chain on lane 0, envelope points and cutoffs to the impression's slots.
// Envelope slots of impression i start at iptr[i] + i (deg + 1 entries),
// cutoff slots at iptr[i] + 2 i (deg + 2 entries).
__global__ __launch_bounds__(64) void envelope_kernel(const int64_t* __restrict__ iptr,
                                                      const int32_t* __restrict__ iadv,
                                                      const double* __restrict__ ibid,
                                                      const double* __restrict__ w, double* env_u,
                                                      double* env_v, double* cut, int32_t* hull_h) {
    __shared__ double sc[kDegMax], sp[kDegMax];
    __shared__ int sa[kDegMax], stk[kDegMax];
    const int i = blockIdx.x, lane = threadIdx.x;
    const int64_t b0 = iptr[i], b1 = iptr[i + 1];
    const int deg = (int)(b1 - b0);
    if (deg == 0) {
        if (lane == 0) hull_h[i] = 0;
        return;
    }
    const int n = deg + 1;
    int np2 = 1;
    while (np2 < n) np2 <<= 1;
    for (int t = lane; t < np2; t += 64) {
        if (t < deg) {
            const double p = ibid[b0 + t];
            const int a = iadv[b0 + t];
            sp[t] = p;
            sc[t] = p * w[a];
            sa[t] = a;
        } else if (t == deg) {
            sp[t] = 0.0;
            sc[t] = 0.0;
            sa[t] = -1;
        } else {
            sp[t] = -__builtin_inf();
            sc[t] = -__builtin_inf();
            sa[t] = 0x7fffffff;
        }
    }
    __syncthreads();
    for (int k = 2; k <= np2; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int t = lane; t < np2; t += 64) {
                const int o = t ^ j;
                if (o > t) {
                    const HullPt A{sc[t], sp[t], sa[t]}, B{sc[o], sp[o], sa[o]};
                    const bool asc = (t & k) == 0;   // "ascending" = hull order
                    if (asc ? hull_before(B, A) : hull_before(A, B)) {
                        sc[t] = B.c; sp[t] = B.p; sa[t] = B.adv;
                        sc[o] = A.c; sp[o] = A.p; sa[o] = A.adv;
                    }
                }
            }
            __syncthreads();
        }
    }
    if (lane != 0) return;
    envelope_chain(sc, sp, sa, stk, n, b0, i, env_u, env_v, cut, hull_h);
}

// Several impressions per 64-lane workgroup (SEG lanes each, every impression
// with deg + 1 <= SEG points): the same total-order sort (SEG-element bitonic
// network, padding last) and the same chain, run by lane 0 of each segment.
template <int SEG>
__global__ __launch_bounds__(64) void envelope_seg_kernel(const int64_t* __restrict__ iptr,
                                                          const int32_t* __restrict__ iadv,
                                                          const double* __restrict__ ibid,
                                                          const double* __restrict__ w, int I, double* env_u,
                                                          double* env_v, double* cut, int32_t* hull_h) {
    __shared__ double sc_all[64], sp_all[64];
    __shared__ int sa_all[64], stk_all[64];
    const int lane = threadIdx.x, sg = lane / SEG, t = lane % SEG;
    const int i = blockIdx.x * (64 / SEG) + sg;
    double* sc = sc_all + sg * SEG;
    double* sp = sp_all + sg * SEG;
    int* sa = sa_all + sg * SEG;
    int64_t b0 = 0;
    int deg = 0;
    if (i < I) {
        b0 = iptr[i];
        deg = (int)(iptr[i + 1] - b0);
    }
    if (t < deg) {
        const double p = ibid[b0 + t];
        const int a = iadv[b0 + t];
        sp[t] = p;
        sc[t] = p * w[a];
        sa[t] = a;
    } else if (t == deg) {
        sp[t] = 0.0;
        sc[t] = 0.0;
        sa[t] = -1;
    } else {
        sp[t] = -__builtin_inf();
        sc[t] = -__builtin_inf();
        sa[t] = 0x7fffffff;
    }
    __syncthreads();
    for (int k = 2; k <= SEG; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            const int o = t ^ j;
            if (o > t) {
                const HullPt A{sc[t], sp[t], sa[t]}, B{sc[o], sp[o], sa[o]};
                const bool asc = (t & k) == 0;
                if (asc ? hull_before(B, A) : hull_before(A, B)) {
                    sc[t] = B.c; sp[t] = B.p; sa[t] = B.adv;
                    sc[o] = A.c; sp[o] = A.p; sa[o] = A.adv;
                }
            }
            __syncthreads();
        }
    }
    if (t != 0 || i >= I) return;
    if (deg == 0) {
        hull_h[i] = 0;
        return;
    }
    envelope_chain(sc, sp, sa, stk_all + sg * SEG, deg + 1, b0, i, env_u, env_v, cut, hull_h);
}

__global__ void region_count_kernel(const int32_t* __restrict__ hull_h, int I, int32_t* cnt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < I) cnt[i] = hull_h[i] >= 2 ? hull_h[i] - 1 : 0;
}

// Regions in (impression asc, region asc) order: key = slope u_j, value = id.
__global__ void emit_regions_kernel(const int64_t* __restrict__ iptr, const int32_t* __restrict__ hull_h,
                                    const int32_t* __restrict__ roff, const double* __restrict__ env_u,
                                    const double* __restrict__ cut, int I, double* keys, int32_t* ids,
                                    int32_t* reg_imp, int32_t* reg_j, double* rwidth) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= I) return;
    const int h = hull_h[i];
    const int64_t bu = iptr[i] + i, bc = iptr[i] + 2 * (int64_t)i;
    for (int j = 0; j + 1 < h; ++j) {
        const int id = roff[i] + j;
        keys[id] = env_u[bu + j];
        ids[id] = id;
        reg_imp[id] = i;
        reg_j[id] = j;
        if (rwidth) rwidth[id] = cut[bc + j + 1] - cut[bc + j];
    }
}

// Chunked budget prefix (spec): chunk sums of the region widths in sorted order.
__global__ void chunk_sum_kernel(const int32_t* __restrict__ sorted_ids, const int32_t* __restrict__ reg_imp,
                                 const int32_t* __restrict__ reg_j, const int64_t* __restrict__ iptr,
                                 const double* __restrict__ cut, int64_t R, double* __restrict__ width,
                                 double* __restrict__ chunk) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t k0 = c * kChunk;
    if (k0 >= R) return;
    const int64_t k1 = (k0 + kChunk < R) ? k0 + kChunk : R;
    double acc = 0.0;
    for (int64_t k = k0; k < k1; ++k) {
        const int id = sorted_ids[k];
        const int i = reg_imp[id], j = reg_j[id];
        const int64_t bc = iptr[i] + 2 * (int64_t)i;
        const double wd = cut[bc + j + 1] - cut[bc + j];
        width[k] = wd;
        acc = acc + wd;
    }
    chunk[c] = acc;
}

__global__ void chunk_offset_kernel(const double* __restrict__ chunk, int64_t nch,
                                    double* __restrict__ offs) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double off = 0.0;
    for (int64_t c = 0; c < nch; ++c) {
        offs[c] = off;
        off = off + chunk[c];
    }
}

__global__ void allocate_kernel(const int32_t* __restrict__ sorted_ids, const double* __restrict__ width,
                                const double* __restrict__ offs, const double* __restrict__ Bptr,
                                int64_t R, double* __restrict__ inc_by_id, int32_t* __restrict__ pos_by_id) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t k0 = c * kChunk;
    if (k0 >= R) return;
    const int64_t k1 = (k0 + kChunk < R) ? k0 + kChunk : R;
    const double B = *Bptr;
    double acc = offs[c];
    for (int64_t k = k0; k < k1; ++k) {
        const double pre = acc;
        const double wd = width[k];
        acc = acc + wd;
        double rem = B - pre;
        if (!(rem > 0.0)) rem = 0.0;
        const int id = sorted_ids[k];
        inc_by_id[id] = (wd < rem) ? wd : rem;   // std::min(rem, width)
        pos_by_id[id] = (int32_t)k;
    }
}

// Primal construction + dual contribution, one lane per impression.
__global__ void primal_kernel(const int64_t* __restrict__ iptr, const int32_t* __restrict__ iadv,
                              const double* __restrict__ ibid, const double* __restrict__ w,
                              const int32_t* __restrict__ hull_h, const int32_t* __restrict__ roff,
                              const double* __restrict__ env_u, const double* __restrict__ env_v,
                              const double* __restrict__ inc_by_id, const int32_t* __restrict__ pos_by_id,
                              int I, double tight_tol, int binary, double* __restrict__ x,
                              double* __restrict__ dcontrib) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= I) return;
    const int64_t b0 = iptr[i], b1 = iptr[i + 1];
    for (int64_t q = b0; q < b1; ++q) x[q] = 0.0;
    dcontrib[i] = 0.0;
    const int h = hull_h[i];
    if (h < 2) return;
    double beta = 0.0;
    int jstar = -1;
    if (binary) {
        // binary mode: pos_by_id holds the region state (1 full, 2 tie); full
        // regions first, then ties, each in region order (R/global_problem.cpp:166-221)
        for (int pass = 1; pass <= 2; ++pass)
            for (int j = 0; j < h - 1; ++j)
                if (pos_by_id[roff[i] + j] == pass) {
                    beta = beta + inc_by_id[roff[i] + j];
                    jstar = j;
                }
    }
    // sort mode: visit this impression's regions in global sorted order
    int last = -1;
    for (int step = 0; !binary && step < h - 1; ++step) {
        int best = -1, bpos = 0x7fffffff;
        for (int j = 0; j < h - 1; ++j) {
            const int pos = pos_by_id[roff[i] + j];
            if (pos > last && pos < bpos) { bpos = pos; best = j; }
        }
        last = bpos;
        const double inc = inc_by_id[roff[i] + best];
        if (inc > 0.0) {
            beta = beta + inc;
            jstar = best;
        }
    }
    if (!(beta > 0.0)) return;
    const int64_t bu = b0 + i;
    const double u = env_u[bu + jstar], v = env_v[bu + jstar];
    const double t0 = u * beta;
    dcontrib[i] = t0 + v;
    if (u == 0.0) {   // greedy by price
        int64_t best = -1;
        double mp = 0.0;
        for (int64_t q = b0; q < b1; ++q)
            if (mp < ibid[q]) { mp = ibid[q]; best = q; }
        if (best >= 0) x[best] = 1.0;
    }
    if (v == 0.0) {   // greedy by price / coefficient
        int64_t best = -1;
        double mr = 0.0;
        for (int64_t q = b0; q < b1; ++q) {
            const double c = ibid[q] * w[iadv[q]];
            const double r = ibid[q] / c;
            if (mr < r) { mr = r; best = q; }
        }
        if (best >= 0) x[best] = beta / (ibid[best] * w[iadv[best]]);
    }
    if (u > 0.0 && v > 0.0) {   // the (at most two) tight constraints
        int64_t q0 = -1, q1 = -1;
        int nt = 0;
        for (int64_t q = b0; q < b1; ++q) {
            const double c = ibid[q] * w[iadv[q]];
            const double uc = u * c;
            double sl = ibid[q] - (uc + v);
            if (sl < 0) sl = -sl;
            if (sl < tight_tol) {
                if (nt == 0) q0 = q; else if (nt == 1) q1 = q;
                ++nt;
            }
        }
        if (nt == 1) {
            const double c = ibid[q0] * w[iadv[q0]];
            x[q0] = __builtin_fmin(beta / c, 1.0);
        } else if (nt == 2) {
            const double c0 = ibid[q0] * w[iadv[q0]], c1 = ibid[q1] * w[iadv[q1]];
            const double x1 = (beta - c1) / (c0 - c1);
            x[q0] = x1;
            x[q1] = 1.0 - x1;
        }
    }
}

__global__ void average_kernel(const double* __restrict__ x, double* __restrict__ xa, int64_t nnz,
                               double fa, double fb) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < nnz) {
        const double a = fa * xa[q], b = fb * x[q];
        xa[q] = a + b;
    }
}

// Per advertiser: slack (impressions ascending), running average, weight.
__global__ void advertiser_kernel(const int64_t* __restrict__ aptr, const int64_t* __restrict__ apos,
                                  const double* __restrict__ abid, const double* __restrict__ budgets,
                                  const double* __restrict__ x, int A, double fa, double fb,
                                  double width, double lp, double lm, double* __restrict__ slack,
                                  double* __restrict__ avg_slack, double* __restrict__ w) {
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= A) return;
    double s = -budgets[a];
    for (int64_t k = aptr[a]; k < aptr[a + 1]; ++k) {
        const double t = x[apos[k]] * abid[k];
        s = s + t;
    }
    slack[a] = s;
    const double p = fa * avg_slack[a], q = fb * s;
    avg_slack[a] = p + q;
    const double tt = s / width;
    const double f = (tt >= 0.0) ? dexp(tt * lp) : dexp(-tt * lm);
    w[a] = w[a] * f;
}

struct BinState;
__device__ inline int bin_levels(const BinState* st);

// Per-iteration report: worst average infeasibility (first index on ties),
// min / max weight; writes log[t].  Every combine is exact (max with a first-
// index tie rule, fmin, fmax), so blocks of 256 lanes reduce in any order;
// the block that finishes last combines the block partials.
struct ReportPart {
    double worst, mn, mx;
    int32_t wi, pad;
};

__device__ inline void report_combine(double& worst, int& wi, double& mn, double& mx, double ow, int oi,
                                      double omn, double omx) {
    if (ow > worst || (ow == worst && oi >= 0 && (wi < 0 || oi < wi))) {
        worst = ow;
        wi = oi;
    }
    mn = __builtin_fmin(mn, omn);
    mx = __builtin_fmax(mx, omx);
}

__device__ inline void report_wave(double& worst, int& wi, double& mn, double& mx) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
        report_combine(worst, wi, mn, mx, __shfl_xor(worst, m), __shfl_xor(wi, m), __shfl_xor(mn, m),
                       __shfl_xor(mx, m));
}

__global__ __launch_bounds__(256) void report_kernel(const double* __restrict__ avg_slack,
                                                     const double* __restrict__ budgets,
                                                     const double* __restrict__ w, int A,
                                                     const double* __restrict__ dual,
                                                     const double* __restrict__ Bptr,
                                                     const BinState* __restrict__ bst, ReportPart* part,
                                                     uint32_t* ticket, dlp_mw_iter* __restrict__ log) {
    __shared__ ReportPart sp[4];
    __shared__ int last;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double worst = 0.0, mn = 100000.0, mx = 0.0;   // R/allocation_mw.cpp:254-255
    int wi = -1;
    for (int a = blockIdx.x * 256 + tid; a < A; a += gridDim.x * 256) {
        const double s = avg_slack[a];
        if (s > 0.0) {
            const double r = s / budgets[a];
            if (r > worst) { worst = r; wi = a; }
        }
        mn = __builtin_fmin(mn, w[a]);
        mx = __builtin_fmax(mx, w[a]);
    }
    report_wave(worst, wi, mn, mx);
    if (lane == 0) sp[wv] = ReportPart{worst, mn, mx, wi, 0};
    __syncthreads();
    if (tid == 0) {
        for (int k = 1; k < 4; ++k) report_combine(worst, wi, mn, mx, sp[k].worst, sp[k].wi, sp[k].mn, sp[k].mx);
        part[blockIdx.x] = ReportPart{worst, mn, mx, wi, 0};
        __threadfence();
        last = (atomicAdd(ticket, 1u) == gridDim.x - 1);
    }
    __syncthreads();
    if (!last || wv != 0) return;
    __threadfence();
    worst = 0.0; mn = 100000.0; mx = 0.0; wi = -1;
    for (int b = lane; b < (int)gridDim.x; b += 64) {
        const ReportPart q = part[b];
        report_combine(worst, wi, mn, mx, q.worst, q.wi, q.mn, q.mx);
    }
    report_wave(worst, wi, mn, mx);
    if (lane == 0) {
        dlp_mw_iter e;
        e.dual_value = *dual;
        e.max_infeasibility = worst;
        e.infeasible_advertiser = wi;
        e.search_levels = bst ? bin_levels(bst) : 0;
        e.min_weight = mn;
        e.max_weight = mx;
        e.weighted_budget = *Bptr;
        *log = e;
        *ticket = 0;
    }
}

// ---------------------------------------------------------------- binary mode
constexpr int kBinMaxRatios = 8;      // num_bin_intervals accepted (the reference uses 3)
constexpr int kBinMaxLevels = 2048;   // spec: level cap
constexpr int kBinBlock = 256;        // spec: block of the blocked sum
constexpr int kBinSingleBlocks = 64;  // whole search in one workgroup up to 64 x 256 impressions

// Search state, device resident across levels (R/global_problem.cpp:46-53).
struct BinState {
    double lower, upper;
    double cr[kBinMaxRatios];
    double S[kBinMaxRatios];          // usage at the last level's ratios (diagnostic)
    double fin_lo, fin_up;            // final interval, (cr, cr) on an exact hit
    double slope_lo, slope_hi;        // FindMinMaxSlope, iteration 1 only
    double rem;                       // budget left for the tie regions
    int32_t nr, levels, done, mode;   // mode 1 = exact ratio, 2 = range
    int32_t pad;
};

__device__ inline int bin_levels(const BinState* st) { return st->levels; }

// Critical ratios of a level: ratio = lower - d, cr_k = (ratio += d)  R/global_problem.cpp:55-62
__device__ inline void bin_set_ratios(BinState* st) {
    const int nr = st->nr;
    const double d = (st->upper - st->lower) / (double)nr;
    double r = st->lower - d;
    for (int k = 0; k < nr; ++k) {
        r = r + d;
        st->cr[k] = r;
    }
}

// The reference's bracket / expand / exact rule after one level
// (R/global_problem.cpp:66-111) and the spec's fp64 stop.  One thread.
__device__ inline void bin_control(BinState* st, const double* S, double B) {
    const int nr = st->nr;
    double lower = st->lower, upper = st->upper;
    st->levels += 1;
    for (int k = 0; k < nr; ++k) st->S[k] = S[k];
    bool expanded = false;
    int exact = -1;
    for (int k = 0; k < nr; ++k) {
        const double delta = S[k] - B;
        if (k == 0 && delta < 0.0) { lower = lower * 0.9; expanded = true; break; }
        if (k == nr - 1 && delta > 0.0) { upper = upper / 0.9; expanded = true; break; }
        if (delta > 0.0) lower = st->cr[k];
        else if (delta < 0.0) { upper = st->cr[k]; break; }
        else { exact = k; break; }
    }
    if (exact >= 0) {
        st->mode = 1;
        st->fin_lo = st->fin_up = st->cr[exact];
        st->done = 1;
        return;
    }
    st->lower = lower;
    st->upper = upper;
    const double a = __builtin_fabs(upper) * 0x1p-42;
    const double tol = (1e-16 < a) ? a : 1e-16;   // std::max(1e-16, |upper| 2^-42)
    if ((!expanded && upper - lower < tol) || st->levels >= kBinMaxLevels) {
        st->mode = 2;
        st->fin_lo = lower;
        st->fin_up = upper;
        st->done = 1;
        return;
    }
    bin_set_ratios(st);
}

// usage_i(cr_k) = sum over the impression's regions (in order) of width if
// u >= cr_k, for the n regions at r0 of ku (slopes) / kw (widths).
__device__ inline void bin_usage_rn(int r0, int n, const double* ku, const double* kw, const double* cr, int nr,
                                    double* acc) {
#pragma unroll
    for (int k = 0; k < kBinMaxRatios; ++k) acc[k] = 0.0;
    // loads issued 4 regions ahead of the (ordered) conditional adds
    constexpr int U = 4;
    for (int j0 = 0; j0 < n; j0 += U) {
        double u[U], w[U];
#pragma unroll
        for (int q = 0; q < U; ++q) {
            const int j = (j0 + q < n) ? j0 + q : n - 1;
            u[q] = ku[r0 + j];
            w[q] = kw[r0 + j];
        }
#pragma unroll
        for (int q = 0; q < U; ++q) {
            if (j0 + q >= n) break;
#pragma unroll
            for (int k = 0; k < kBinMaxRatios; ++k)
                if (k < nr && u[q] >= cr[k]) acc[k] = acc[k] + w[q];
        }
    }
}

__device__ inline void bin_usage(int i, int I, const int32_t* __restrict__ roff,
                                 const int32_t* __restrict__ rcnt, const double* __restrict__ keys,
                                 const double* __restrict__ rwidth, const double* cr, int nr,
                                 double* acc) {
    const bool in = i < I;
    bin_usage_rn(in ? roff[i] : 0, in ? rcnt[i] : 0, keys, rwidth, cr, nr, acc);
}

// Spec block tree over 256 lanes (lds[k][256] filled, synchronised): s_l += s_{l+w},
// w = 128 .. 1; the block sum of row k lands in lane 0 of wave 0 (returned there).
template <int NK>
__device__ inline void bin_block_tree(double (*lds)[kBinBlock], int nk, int tid, double* out) {
    if (tid < 128)
        for (int k = 0; k < nk; ++k) lds[k][tid] = lds[k][tid] + lds[k][tid + 128];
    __syncthreads();
    if (tid < 64) {
        for (int k = 0; k < nk; ++k) {
            double x = lds[k][tid] + lds[k][tid + 64];
#pragma unroll
            for (int w = 32; w >= 1; w >>= 1) x = x + __shfl_down(x, w);
            if (tid == 0) out[k] = x;
        }
    }
}

// FindMinMaxSlope (R/global_problem.cpp:116-135) over regions in id order =
// (impression asc, region asc), in chunks of 256: a region is a running-maximum
// record iff it exceeds the maximum before it (initial 0); the minimum runs
// over the non-records only (the reference's else-if).
__global__ void rec_chunk_max_kernel(const double* __restrict__ keys, int64_t R, double* __restrict__ cmax) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t k0 = c * kBinBlock;
    if (k0 >= R) return;
    const int64_t k1 = (k0 + kBinBlock < R) ? k0 + kBinBlock : R;
    double mx = -DBL_MAX;
    for (int64_t k = k0; k < k1; ++k) mx = __builtin_fmax(mx, keys[k]);
    cmax[c] = mx;
}

__global__ void rec_prefix_kernel(const double* __restrict__ cmax, int64_t nch, double* __restrict__ pmax) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    double run = 0.0;   // max_weight = 0.0
    for (int64_t c = 0; c < nch; ++c) {
        pmax[c] = run;
        run = __builtin_fmax(run, cmax[c]);
    }
}

__global__ void rec_chunk_min_kernel(const double* __restrict__ keys, int64_t R,
                                     const double* __restrict__ pmax, double* __restrict__ cmin,
                                     double* __restrict__ cmax) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t k0 = c * kBinBlock;
    if (k0 >= R) return;
    const int64_t k1 = (k0 + kBinBlock < R) ? k0 + kBinBlock : R;
    double run = pmax[c], mn = DBL_MAX;
    for (int64_t k = k0; k < k1; ++k) {
        const double u = keys[k];
        if (u > run) run = u;
        else if (u < mn) mn = u;
    }
    cmin[c] = mn;
    cmax[c] = run;   // running maximum at the chunk's end
}

__global__ __launch_bounds__(64) void rec_final_kernel(const double* __restrict__ cmin,
                                                       const double* __restrict__ cmax, int64_t nch,
                                                       BinState* st) {
    double mn = DBL_MAX, mx = 0.0;
    for (int64_t c = threadIdx.x; c < nch; c += 64) {
        mn = __builtin_fmin(mn, cmin[c]);
        mx = __builtin_fmax(mx, cmax[c]);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        mn = __builtin_fmin(mn, __shfl_xor(mn, m));
        mx = __builtin_fmax(mx, __shfl_xor(mx, m));
    }
    if (threadIdx.x == 0) {
        st->slope_lo = 1.0 / mx;   // min_slope_ = 1 / max_weight
        st->slope_hi = 1.0 / mn;   // max_slope_ = 1 / min_weight
    }
}

// Start of a search: [slope_lo, slope_hi] at iteration 1, [slope_lo*scale,
// slope_hi/scale] after (R/global_problem.cpp:283-292).
__global__ void bin_begin_kernel(BinState* st, int first, double scale, int nr) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    st->lower = first ? st->slope_lo : st->slope_lo * scale;
    st->upper = first ? st->slope_hi : st->slope_hi / scale;
    st->nr = nr;
    st->levels = 0;
    st->done = 0;
    st->mode = 0;
    st->rem = 0.0;
    bin_set_ratios(st);
}

// One search level over all impressions: block sums of the nr usages (spec
// tree per 256 impressions).  A launch after the search stopped returns at
// once.  No cross-block hand-off inside the kernel: a device-scope fence per
// block is an L2 write-back per block on gfx950; the kernel boundary orders
// the block sums for bin_control_kernel instead.
__global__ __launch_bounds__(kBinBlock) void bin_level_kernel(const BinState* st, const int32_t* __restrict__ roff,
                                                              const int32_t* __restrict__ rcnt,
                                                              const double* __restrict__ keys,
                                                              const double* __restrict__ rwidth, int I,
                                                              double* __restrict__ bsum) {
    if (st->done) return;
    __shared__ double lds[kBinMaxRatios][kBinBlock];
    __shared__ double tot[kBinMaxRatios];
    const int nr = st->nr, tid = threadIdx.x, nb = gridDim.x, b = blockIdx.x;
    double cr[kBinMaxRatios], acc[kBinMaxRatios];
#pragma unroll
    for (int k = 0; k < kBinMaxRatios; ++k) cr[k] = (k < nr) ? st->cr[k] : 0.0;
    bin_usage(b * kBinBlock + tid, I, roff, rcnt, keys, rwidth, cr, nr, acc);
#pragma unroll
    for (int k = 0; k < kBinMaxRatios; ++k)
        if (k < nr) lds[k][tid] = acc[k];
    __syncthreads();
    bin_block_tree<kBinMaxRatios>(lds, nr, tid, tot);
    if (tid == 0)
        for (int k = 0; k < nr; ++k) bsum[(int64_t)k * nb + b] = tot[k];
}

// sum_fixed of each ratio's block sums (one wave per ratio) and the control rule.
__global__ __launch_bounds__(kBinBlock) void bin_control_kernel(BinState* st, const double* __restrict__ bsum,
                                                                int nb, const double* __restrict__ Bptr) {
    if (st->done) return;
    __shared__ double tot[kBinMaxRatios];
    const int nr = st->nr, tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    for (int k = wv; k < nr; k += kBinBlock / 64) {
        const double a = wave_sum_fixed(bsum + (int64_t)k * nb, nb, lane);
        if (lane == 0) tot[k] = a;
    }
    __syncthreads();
    if (tid == 0) bin_control(st, tot, *Bptr);
}

// The whole search in one workgroup of 1024 lanes (nb <= kBinSingleBlocks):
// four 256-lane groups take the blocks of the spec in turn; the control state
// lives in LDS.  With at most 4 blocks every lane keeps its impression's
// region range in registers, and the regions (slope, width) are staged in LDS
// once when they fit (`cached`), so a level touches no global memory.
__global__ __launch_bounds__(1024) void bin_search_single_kernel(BinState* st, const int32_t* __restrict__ roff,
                                                                 const int32_t* __restrict__ rcnt,
                                                                 const double* __restrict__ keys,
                                                                 const double* __restrict__ rwidth, int I,
                                                                 int R, int cached,
                                                                 const double* __restrict__ Bptr) {
    extern __shared__ double rcache[];   // 2R doubles when cached
    __shared__ double lds[4][kBinBlock];
    __shared__ double bs[kBinMaxRatios][kBinSingleBlocks];
    __shared__ double tot[kBinMaxRatios];
    __shared__ BinState ss;
    const int tid = threadIdx.x, g = tid >> 8, gl = tid & 255;
    const int nb = (I + kBinBlock - 1) / kBinBlock;
    if (tid == 0) ss = *st;
    if (cached)
        for (int k = tid; k < R; k += 1024) {
            rcache[k] = keys[k];
            rcache[R + k] = rwidth[k];
        }
    const double* ku = cached ? rcache : keys;
    const double* kw = cached ? rcache + R : rwidth;
    const bool one_round = nb <= 4;
    int r0 = 0, n = 0;
    if (one_round && g * kBinBlock + gl < I) {
        r0 = roff[g * kBinBlock + gl];
        n = rcnt[g * kBinBlock + gl];
    }
    __syncthreads();
    const int nr = ss.nr;
    const double B = *Bptr;
    while (!ss.done) {
        double cr[kBinMaxRatios], acc[kBinMaxRatios];
#pragma unroll
        for (int k = 0; k < kBinMaxRatios; ++k) cr[k] = (k < nr) ? ss.cr[k] : 0.0;
        for (int b0 = 0; b0 < nb; b0 += 4) {
            const int b = b0 + g;
            if (!one_round) {
                const int i = b * kBinBlock + gl;
                r0 = (b < nb && i < I) ? roff[i] : 0;
                n = (b < nb && i < I) ? rcnt[i] : 0;
            }
            bin_usage_rn(r0, b < nb ? n : 0, ku, kw, cr, nr, acc);
#pragma unroll
            for (int k = 0; k < kBinMaxRatios; ++k) {
                if (k >= nr) break;
                lds[g][gl] = acc[k];
                __syncthreads();
                if (gl < 128) lds[g][gl] = lds[g][gl] + lds[g][gl + 128];
                __syncthreads();
                if (gl < 64 && b < nb) {
                    double x = lds[g][gl] + lds[g][gl + 64];
#pragma unroll
                    for (int w = 32; w >= 1; w >>= 1) x = x + __shfl_down(x, w);
                    if (gl == 0) bs[k][b] = x;
                }
                __syncthreads();
            }
        }
        const int wv = tid >> 6, lane = tid & 63;
        if (wv < nr) {
            const double a = wave_sum_fixed(bs[wv], nb, lane);
            if (lane == 0) tot[wv] = a;
        }
        __syncthreads();
        if (tid == 0) bin_control(&ss, tot, B);
        __syncthreads();
    }
    if (tid == 0) *st = ss;
}

// Final allocation, full part (R/global_problem.cpp:166-178 exact hit,
// 180-195 range): state 1 + inc = width for regions u >= cr (exact) or
// u > upper (range); tie candidates lower < u <= upper flagged; block sums
// of the full part per impression (spec tree) for bin_rem_kernel.
__global__ __launch_bounds__(kBinBlock) void bin_assign_kernel(const BinState* st, const int32_t* __restrict__ roff,
                                                               const int32_t* __restrict__ rcnt,
                                                               const double* __restrict__ keys,
                                                               const double* __restrict__ rwidth, int I,
                                                               int32_t* __restrict__ rstate,
                                                               double* __restrict__ inc,
                                                               uint8_t* __restrict__ flags,
                                                               double* __restrict__ bsum) {
    __shared__ double lds[1][kBinBlock];
    __shared__ double tot[1];
    const int tid = threadIdx.x, b = blockIdx.x;
    const int i = b * kBinBlock + tid;
    const int mode = st->mode;
    const double lo = st->fin_lo, up = st->fin_up;
    double beta = 0.0;
    if (i < I) {
        const int r0 = roff[i], n = rcnt[i];
        for (int j = 0; j < n; ++j) {
            const double u = keys[r0 + j], w = rwidth[r0 + j];
            const bool full = (mode == 1) ? (u >= lo) : (u > up);
            const bool tie = (mode == 2) && (u > lo) && (u <= up);
            rstate[r0 + j] = full ? 1 : 0;
            inc[r0 + j] = full ? w : 0.0;
            flags[r0 + j] = tie ? 1 : 0;
            if (full) beta = beta + w;
        }
    }
    lds[0][tid] = beta;
    __syncthreads();
    bin_block_tree<1>(lds, 1, tid, tot);
    if (tid == 0) bsum[b] = tot[0];
}

// rem = B - sum_fixed(block sums of the full part).
__global__ __launch_bounds__(64) void bin_rem_kernel(BinState* st, const double* __restrict__ bsum, int nb,
                                                     const double* __restrict__ Bptr) {
    const double a = wave_sum_fixed(bsum, nb, threadIdx.x);
    if (threadIdx.x == 0) st->rem = *Bptr - a;
}

// Tie regions in (impression, region) order (R/global_problem.cpp:197-221):
// inc = min(rem, width), assigned whatever its sign, rem -= inc, stop at
// rem == 0.  rem reaches 0 exactly at the first tie whose width is not below
// the budget left (fl(a - b) == 0 iff a == b), so a batch of 64 runs the
// serial chain r_{k+1} = r_k - w_k alone (one dependent add per tie; r_k
// parked in lane k), then one ballot finds the stopping tie.  One wave.
__global__ __launch_bounds__(64) void bin_tie_chain_kernel(BinState* st, const int32_t* __restrict__ tie_ids,
                                                           const int32_t* __restrict__ num_ties,
                                                           const double* __restrict__ rwidth,
                                                           int32_t* __restrict__ rstate,
                                                           double* __restrict__ inc) {
    const int lane = threadIdx.x;
    const int n = *num_ties;
    double rem = st->rem;
    int serial_from = -1;
    for (int base = 0; base < n; base += 64) {
        const int q = base + lane;
        const int id = (q < n) ? tie_ids[q] : 0;
        const double w = (q < n) ? rwidth[id] : 0.0;
        const int cnt = (n - base < 64) ? n - base : 64;
        const uint64_t wb = __builtin_bit_cast(uint64_t, w);
        const int wlo = (int)(uint32_t)wb, whi = (int)(uint32_t)(wb >> 32);
        double r = 0.0;   // r_lane
        for (int k = 0; k < cnt; ++k) {
            r = (lane == k) ? rem : r;
            const uint64_t kb = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(whi, k) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane(wlo, k);
            rem = rem - __builtin_bit_cast(double, kb);
        }
        const bool stop_here = (lane < cnt) && !(w < r);   // std::min(rem, width) takes rem
        const uint64_t ball = __ballot(stop_here);
        const int f = ball ? __builtin_ctzll(ball) : cnt;
        if (lane < cnt && lane <= f) {
            inc[id] = (lane == f) ? r : w;
            rstate[id] = 2;
        }
        if (ball) {
            const double rf = __shfl(r, f);
            rem = rf - rf;   // 0 unless the budget is not finite
            if (rem != 0.0) serial_from = base + f + 1;
            break;
        }
    }
    // non-finite budget (inf - inf): the literal walk for the rest
    for (int q = serial_from; q >= 0 && q < n; ++q) {
        const int id = tie_ids[q];
        const double w = rwidth[id];
        const double a = (w < rem) ? w : rem;
        if (lane == 0) {
            inc[id] = a;
            rstate[id] = 2;
        }
        rem = rem - a;
        if (rem == 0.0) break;
    }
    if (lane == 0) st->rem = rem;
}

}  // namespace mw
}  // namespace dlp

struct dlp_mw {
    int device = 0;
    hipStream_t stream = nullptr;
    int A = 0, I = 0;
    int64_t nnz = 0;
    double width = 0, lp = 0, lm = 0, tight_tol = 1e-12;
    int t = 0;   // iterations done
    // device arrays
    int64_t *iptr = nullptr, *aptr = nullptr, *apos = nullptr;
    int32_t *iadv = nullptr;
    double *ibid = nullptr, *abid = nullptr, *budgets = nullptr, *w = nullptr, *wb = nullptr;
    double *slack = nullptr, *avg_slack = nullptr, *x = nullptr, *xa = nullptr;
    double *env_u = nullptr, *env_v = nullptr, *cut = nullptr;
    int32_t *hull_h = nullptr, *rcnt = nullptr, *roff = nullptr;
    double *keys = nullptr, *keys_sorted = nullptr, *width_sorted = nullptr;
    int32_t *ids = nullptr, *ids_sorted = nullptr, *reg_imp = nullptr, *reg_j = nullptr, *pos_by_id = nullptr;
    double *inc_by_id = nullptr, *chunk = nullptr, *offs = nullptr, *dcontrib = nullptr;
    double *B = nullptr, *dual = nullptr;
    int32_t *rtotal = nullptr;
    dlp_mw_iter* dlog = nullptr;
    int log_cap = 0;
    // binary mode
    int maxdeg = 0;
    int binary = 0, nr = 3;
    double scale = 0.0;
    double *rwidth = nullptr, *bsum = nullptr, *cmax = nullptr, *pmax = nullptr, *cmin = nullptr;
    uint8_t* flags = nullptr;
    int32_t *tie_ids = nullptr, *num_ties = nullptr;
    dlp::mw::BinState* bst = nullptr;
    dlp::mw::ReportPart* rpart = nullptr;
    uint32_t* rticket = nullptr;
    int report_blocks = 1;
    void* cub_tmp = nullptr;
    size_t cub_bytes = 0;
    std::vector<int64_t> var_to_imp;   // problem variable k -> impression-major index
};

namespace {
using dlp::set_error;

#define MW_TRY(expr)                                                                   \
    do {                                                                               \
        hipError_t e_ = (expr);                                                        \
        if (e_ != hipSuccess) {                                                        \
            set_error(std::string(#expr) + ": " + hipGetErrorString(e_));              \
            return DLP_ERR_HIP;                                                        \
        }                                                                              \
    } while (0)

template <typename T>
int dalloc(T** p, size_t n) {
    if (hipMalloc((void**)p, sizeof(T) * std::max<size_t>(n, 1)) != hipSuccess) {
        set_error("dlp_mw: hipMalloc failed");
        return DLP_ERR_OOM;
    }
    return DLP_OK;
}

void mw_free(dlp_mw* m) {
    if (!m) return;
    (void)hipSetDevice(m->device);
    if (m->stream) (void)hipStreamSynchronize(m->stream);
    void* ptrs[] = {m->iptr, m->aptr, m->apos, m->iadv, m->ibid, m->abid, m->budgets, m->w, m->wb,
                    m->slack, m->avg_slack, m->x, m->xa, m->env_u, m->env_v, m->cut, m->hull_h,
                    m->rcnt, m->roff, m->keys, m->keys_sorted, m->width_sorted, m->ids,
                    m->ids_sorted, m->reg_imp, m->reg_j, m->pos_by_id, m->inc_by_id, m->chunk,
                    m->offs, m->dcontrib, m->B, m->dual, m->rtotal, m->dlog, m->cub_tmp,
                    m->rwidth, m->bsum, m->cmax, m->pmax, m->cmin, m->flags, m->tie_ids,
                    m->num_ties, m->bst, m->rpart, m->rticket};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (m->stream) (void)hipStreamDestroy(m->stream);
    delete m;
}

int mw_init(const dlp_problem* prob, const dlp_mw_options* o, dlp_mw* m) {
    const auto& ad = prob->ad;
    m->device = o->device;
    m->A = ad.num_advertisers;
    m->I = ad.num_impressions;
    m->nnz = (int64_t)ad.adv.size();
    const int A = m->A, I = m->I;
    const int64_t nnz = m->nnz;
    // impression-major order (impression asc, advertiser asc); problem variables are (a asc, i asc)
    std::vector<int64_t> order(nnz);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(),
                     [&](int64_t a, int64_t b) { return ad.imp[a] < ad.imp[b]; });
    std::vector<int64_t> iptr(I + 1, 0), aptr(A + 1, 0), apos(nnz);
    std::vector<int32_t> iadv(nnz);
    std::vector<double> ibid(nnz);
    m->var_to_imp.resize(nnz);
    for (int64_t k = 0; k < nnz; ++k) {
        iptr[ad.imp[k] + 1]++;
        aptr[ad.adv[k] + 1]++;
    }
    for (int i = 0; i < I; ++i) iptr[i + 1] += iptr[i];
    for (int a = 0; a < A; ++a) aptr[a + 1] += aptr[a];
    int maxdeg = 0;
    for (int i = 0; i < I; ++i) maxdeg = std::max<int>(maxdeg, (int)(iptr[i + 1] - iptr[i]));
    m->maxdeg = maxdeg;
    if (maxdeg + 1 > dlp::mw::kDegMax) {
        set_error("dlp_mw: an impression has more bids than the envelope kernel holds");
        return DLP_ERR_UNSUPPORTED;
    }
    for (int64_t q = 0; q < nnz; ++q) {
        const int64_t k = order[q];
        iadv[q] = ad.adv[k];
        ibid[q] = ad.bid[k];
        m->var_to_imp[k] = q;
    }
    for (int64_t k = 0; k < nnz; ++k) apos[k] = m->var_to_imp[k];   // advertiser-major = variable order
    // width R/allocation_mw.cpp:154-161
    double width = ad.max_bid * ((double)I * ad.sparsity);
    for (int a = 0; a < A; ++a) width = std::max(width, ad.budget[a]);
    m->width = width;
    m->lp = std::log1p(o->epsilon);
    m->lm = std::log1p(-o->epsilon);
    m->tight_tol = std::max(o->tolerance, 1e-12);

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_error("no HIP device visible (libdlp has no CPU fallback)");
        return DLP_ERR_NODEVICE;
    }
    MW_TRY(hipSetDevice(m->device));
    MW_TRY(hipStreamCreateWithFlags(&m->stream, hipStreamNonBlocking));
    int rc = DLP_OK;
#define MW_ALLOC(ptr, n) if ((rc = dalloc(&(ptr), (n))) != DLP_OK) return rc
    MW_ALLOC(m->iptr, I + 1); MW_ALLOC(m->aptr, A + 1); MW_ALLOC(m->apos, nnz);
    MW_ALLOC(m->iadv, nnz); MW_ALLOC(m->ibid, nnz); MW_ALLOC(m->abid, nnz);
    MW_ALLOC(m->budgets, A); MW_ALLOC(m->w, A); MW_ALLOC(m->wb, A);
    MW_ALLOC(m->slack, A); MW_ALLOC(m->avg_slack, A); MW_ALLOC(m->x, nnz); MW_ALLOC(m->xa, nnz);
    MW_ALLOC(m->env_u, nnz + I); MW_ALLOC(m->env_v, nnz + I); MW_ALLOC(m->cut, nnz + 2 * (int64_t)I);
    MW_ALLOC(m->hull_h, I); MW_ALLOC(m->rcnt, I); MW_ALLOC(m->roff, I);
    MW_ALLOC(m->keys, nnz); MW_ALLOC(m->keys_sorted, nnz); MW_ALLOC(m->width_sorted, nnz);
    MW_ALLOC(m->ids, nnz); MW_ALLOC(m->ids_sorted, nnz); MW_ALLOC(m->reg_imp, nnz);
    MW_ALLOC(m->reg_j, nnz); MW_ALLOC(m->pos_by_id, nnz); MW_ALLOC(m->inc_by_id, nnz);
    MW_ALLOC(m->chunk, nnz / dlp::mw::kChunk + 2); MW_ALLOC(m->offs, nnz / dlp::mw::kChunk + 2);
    MW_ALLOC(m->dcontrib, I); MW_ALLOC(m->B, 1); MW_ALLOC(m->dual, 1); MW_ALLOC(m->rtotal, 1);
    m->report_blocks = std::max(1, std::min(1024, (A + 255) / 256));
    MW_ALLOC(m->rpart, m->report_blocks); MW_ALLOC(m->rticket, 1);
    MW_TRY(hipMemset(m->rticket, 0, sizeof(uint32_t)));
    m->binary = o->binary ? 1 : 0;
    if (m->binary) {
        using dlp::mw::kBinBlock;
        using dlp::mw::kBinMaxRatios;
        m->nr = o->intervals;
        // R/main.cpp:38: cr_transition_scale = 1 - epsilon * 0.001 (x87 long double), unless given
        m->scale = (o->scale > 0.0) ? o->scale
                                    : (double)(1.0L - (long double)o->epsilon * (long double)0.001);
        const int64_t nb = (I + kBinBlock - 1) / kBinBlock, nch = nnz / kBinBlock + 2;
        MW_ALLOC(m->rwidth, nnz); MW_ALLOC(m->bsum, kBinMaxRatios * nb); MW_ALLOC(m->flags, nnz);
        MW_ALLOC(m->tie_ids, nnz); MW_ALLOC(m->num_ties, 1);
        MW_ALLOC(m->cmax, nch); MW_ALLOC(m->pmax, nch); MW_ALLOC(m->cmin, nch);
        MW_ALLOC(m->bst, 1);
        MW_TRY(hipMemset(m->bst, 0, sizeof(dlp::mw::BinState)));
    }
#undef MW_ALLOC
    std::vector<double> ones(A, 1.0), zeros_a(A, 0.0), zeros_n(nnz, 0.0);
    MW_TRY(hipMemcpy(m->iptr, iptr.data(), sizeof(int64_t) * (I + 1), hipMemcpyHostToDevice));
    MW_TRY(hipMemcpy(m->aptr, aptr.data(), sizeof(int64_t) * (A + 1), hipMemcpyHostToDevice));
    MW_TRY(hipMemcpy(m->apos, apos.data(), sizeof(int64_t) * nnz, hipMemcpyHostToDevice));
    MW_TRY(hipMemcpy(m->iadv, iadv.data(), sizeof(int32_t) * nnz, hipMemcpyHostToDevice));
    MW_TRY(hipMemcpy(m->ibid, ibid.data(), sizeof(double) * nnz, hipMemcpyHostToDevice));
    MW_TRY(hipMemcpy(m->abid, ad.bid.data(), sizeof(double) * nnz, hipMemcpyHostToDevice));
    MW_TRY(hipMemcpy(m->budgets, ad.budget.data(), sizeof(double) * A, hipMemcpyHostToDevice));
    MW_TRY(hipMemcpy(m->w, ones.data(), sizeof(double) * A, hipMemcpyHostToDevice));
    MW_TRY(hipMemcpy(m->slack, zeros_a.data(), sizeof(double) * A, hipMemcpyHostToDevice));
    MW_TRY(hipMemcpy(m->avg_slack, zeros_a.data(), sizeof(double) * A, hipMemcpyHostToDevice));
    MW_TRY(hipMemcpy(m->xa, zeros_n.data(), sizeof(double) * nnz, hipMemcpyHostToDevice));
    MW_TRY(hipMemcpy(m->x, zeros_n.data(), sizeof(double) * nnz, hipMemcpyHostToDevice));
    // hipCUB temporary storage: region sort (<= nnz items) and the region-count scan
    size_t b1 = 0, b2 = 0;
    MW_TRY(hipcub::DeviceRadixSort::SortPairsDescending(nullptr, b1, m->keys, m->keys_sorted, m->ids,
                                                       m->ids_sorted, (int)std::max<int64_t>(nnz, 1),
                                                       0, 64, m->stream));
    MW_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, b2, m->rcnt, m->roff, std::max(I, 1), m->stream));
    size_t b3 = 0;
    if (m->binary)
        MW_TRY(hipcub::DeviceSelect::Flagged(nullptr, b3, hipcub::CountingInputIterator<int32_t>(0), m->flags,
                                             m->tie_ids, m->num_ties, (int)std::max<int64_t>(nnz, 1),
                                             m->stream));
    m->cub_bytes = std::max(std::max(b1, b2), b3);
    MW_TRY(hipMalloc(&m->cub_tmp, std::max<size_t>(m->cub_bytes, 16)));
    return DLP_OK;
}

// Binary-mode budget split (R/global_problem.cpp:46-222, 283-292): the search,
// then the full / tie allocation into inc_by_id + region states (pos_by_id).
int bin_allocate(dlp_mw* m, int64_t R, int t) {
    using namespace dlp::mw;
    hipStream_t s = m->stream;
    const int I = m->I;
    const int nb = (I + kBinBlock - 1) / kBinBlock;
    if (t == 1) {   // FindMinMaxSlope
        const int64_t nch = (R + kBinBlock - 1) / kBinBlock;
        const unsigned g = (unsigned)((nch + 255) / 256);
        if (nch > 0) {
            rec_chunk_max_kernel<<<g, 256, 0, s>>>(m->keys, R, m->cmax);
            rec_prefix_kernel<<<1, 64, 0, s>>>(m->cmax, nch, m->pmax);
            rec_chunk_min_kernel<<<g, 256, 0, s>>>(m->keys, R, m->pmax, m->cmin, m->cmax);
        }
        rec_final_kernel<<<1, 64, 0, s>>>(m->cmin, m->cmax, nch, m->bst);
    }
    bin_begin_kernel<<<1, 64, 0, s>>>(m->bst, t == 1 ? 1 : 0, m->scale, m->nr);
    if (nb <= kBinSingleBlocks) {
        constexpr size_t kCacheMax = 144 * 1024;   // LDS for the region cache (static part ~12.5 KB)
        static bool attr_set[64] = {};
        if (!attr_set[m->device & 63]) {
            MW_TRY(hipFuncSetAttribute((const void*)bin_search_single_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kCacheMax));
            attr_set[m->device & 63] = true;
        }
        // DLP_MW_NO_LDS_CACHE=1: regions read from HBM every level (test knob)
        const char* nc = std::getenv("DLP_MW_NO_LDS_CACHE");
        const bool allow = !(nc && nc[0] == '1');
        const int cached = (allow && R > 0 && (size_t)R * 16 <= kCacheMax) ? 1 : 0;
        bin_search_single_kernel<<<1, 1024, cached ? (size_t)R * 16 : 0, s>>>(
            m->bst, m->roff, m->rcnt, m->keys, m->rwidth, I, (int)R, cached, m->B);
    } else {
        int32_t done = 0;
        for (int issued = 0; !done;) {
            const int batch = issued == 0 ? 48 : 32;
            for (int k = 0; k < batch; ++k) {
                bin_level_kernel<<<nb, kBinBlock, 0, s>>>(m->bst, m->roff, m->rcnt, m->keys, m->rwidth, I,
                                                          m->bsum);
                bin_control_kernel<<<1, kBinBlock, 0, s>>>(m->bst, m->bsum, nb, m->B);
            }
            issued += batch;
            MW_TRY(hipGetLastError());
            MW_TRY(hipMemcpyAsync(&done, &m->bst->done, sizeof(int32_t), hipMemcpyDeviceToHost, s));
            MW_TRY(hipStreamSynchronize(s));
            if (!done && issued > kBinMaxLevels + 64) {
                set_error("dlp_mw: binary search did not stop within the level cap");
                return DLP_ERR_STATE;
            }
        }
    }
    bin_assign_kernel<<<nb, kBinBlock, 0, s>>>(m->bst, m->roff, m->rcnt, m->keys, m->rwidth, I, m->pos_by_id,
                                               m->inc_by_id, m->flags, m->bsum);
    bin_rem_kernel<<<1, 64, 0, s>>>(m->bst, m->bsum, nb, m->B);
    if (R > 0) {
        size_t bytes = m->cub_bytes;
        MW_TRY(hipcub::DeviceSelect::Flagged(m->cub_tmp, bytes, hipcub::CountingInputIterator<int32_t>(0),
                                             m->flags, m->tie_ids, m->num_ties, (int)R, s));
        bin_tie_chain_kernel<<<1, 64, 0, s>>>(m->bst, m->tie_ids, m->num_ties, m->rwidth, m->pos_by_id,
                                              m->inc_by_id);
    }
    MW_TRY(hipGetLastError());
    return DLP_OK;
}

int mw_iteration(dlp_mw* m, dlp_mw_iter* dlog_entry) {
    using namespace dlp::mw;
    const int A = m->A, I = m->I;
    const int64_t nnz = m->nnz;
    hipStream_t s = m->stream;
    const int tb = 256;
    const int t = m->t + 1;
    const double fa = (double)(t - 1) / (double)t, fb = 1.0 / (double)t;
    weighted_budget_kernel<<<(A + tb - 1) / tb, tb, 0, s>>>(m->w, m->budgets, A, m->wb);
    sum_fixed_kernel<<<1, 64, 0, s>>>(m->wb, A, m->B);
    if (m->maxdeg + 1 <= 16)
        envelope_seg_kernel<16><<<(I + 3) / 4, 64, 0, s>>>(m->iptr, m->iadv, m->ibid, m->w, I, m->env_u,
                                                         m->env_v, m->cut, m->hull_h);
    else if (m->maxdeg + 1 <= 32)
        envelope_seg_kernel<32><<<(I + 1) / 2, 64, 0, s>>>(m->iptr, m->iadv, m->ibid, m->w, I, m->env_u,
                                                         m->env_v, m->cut, m->hull_h);
    else
        envelope_kernel<<<I, 64, 0, s>>>(m->iptr, m->iadv, m->ibid, m->w, m->env_u, m->env_v, m->cut,
                                         m->hull_h);
    region_count_kernel<<<(I + tb - 1) / tb, tb, 0, s>>>(m->hull_h, I, m->rcnt);
    size_t bytes = m->cub_bytes;
    MW_TRY(hipcub::DeviceScan::ExclusiveSum(m->cub_tmp, bytes, m->rcnt, m->roff, I, s));
    emit_regions_kernel<<<(I + tb - 1) / tb, tb, 0, s>>>(m->iptr, m->hull_h, m->roff, m->env_u, m->cut,
                                                         I, m->keys, m->ids, m->reg_imp, m->reg_j,
                                                         m->rwidth);
    // region count R = roff[I-1] + rcnt[I-1]: read back (the sort needs it on the host)
    int32_t last[2] = {0, 0};
    MW_TRY(hipMemcpyAsync(&last[0], m->roff + (I - 1), sizeof(int32_t), hipMemcpyDeviceToHost, s));
    MW_TRY(hipMemcpyAsync(&last[1], m->rcnt + (I - 1), sizeof(int32_t), hipMemcpyDeviceToHost, s));
    MW_TRY(hipStreamSynchronize(s));
    const int64_t R = (int64_t)last[0] + last[1];
    if (m->binary) {
        int rc = bin_allocate(m, R, t);
        if (rc != DLP_OK) return rc;
    } else if (R > 0) {
        bytes = m->cub_bytes;
        MW_TRY(hipcub::DeviceRadixSort::SortPairsDescending(m->cub_tmp, bytes, m->keys, m->keys_sorted,
                                                           m->ids, m->ids_sorted, (int)R, 0, 64, s));
        const int64_t nch = (R + kChunk - 1) / kChunk;
        chunk_sum_kernel<<<(unsigned)((nch + tb - 1) / tb), tb, 0, s>>>(
            m->ids_sorted, m->reg_imp, m->reg_j, m->iptr, m->cut, R, m->width_sorted, m->chunk);
        chunk_offset_kernel<<<1, 64, 0, s>>>(m->chunk, nch, m->offs);
        allocate_kernel<<<(unsigned)((nch + tb - 1) / tb), tb, 0, s>>>(
            m->ids_sorted, m->width_sorted, m->offs, m->B, R, m->inc_by_id, m->pos_by_id);
    }
    primal_kernel<<<(I + tb - 1) / tb, tb, 0, s>>>(m->iptr, m->iadv, m->ibid, m->w, m->hull_h, m->roff,
                                                   m->env_u, m->env_v, m->inc_by_id, m->pos_by_id, I,
                                                   m->tight_tol, m->binary, m->x, m->dcontrib);
    sum_fixed_kernel<<<1, 64, 0, s>>>(m->dcontrib, I, m->dual);
    average_kernel<<<(unsigned)((nnz + tb - 1) / tb), tb, 0, s>>>(m->x, m->xa, nnz, fa, fb);
    advertiser_kernel<<<(A + tb - 1) / tb, tb, 0, s>>>(m->aptr, m->apos, m->abid, m->budgets, m->x, A,
                                                       fa, fb, m->width, m->lp, m->lm, m->slack,
                                                       m->avg_slack, m->w);
    report_kernel<<<m->report_blocks, 256, 0, s>>>(m->avg_slack, m->budgets, m->w, A, m->dual, m->B, m->bst,
                                                   m->rpart, m->rticket, dlog_entry);
    MW_TRY(hipGetLastError());
    m->t = t;
    return DLP_OK;
}

}  // namespace

extern "C" {

void dlp_mw_options_default(dlp_mw_options* o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->device = 0;
    o->binary = 0;
    o->epsilon = 0.01;
    o->tolerance = 1e-18;
    o->scale = 0.0;       // derived: 1 - epsilon * 0.001 (R/main.cpp:38)
    o->intervals = 3;     // R/main.cpp:37
}

int dlp_mw_create(const dlp_problem* prob, const dlp_mw_options* opt, dlp_mw** out) {
    dlp_mw_options o;
    if (opt) o = *opt; else dlp_mw_options_default(&o);
    if (!prob || !out || prob->kind != dlp::PROB_ADALLOC || prob->ad.num_impressions <= 0) {
        set_error("dlp_mw_create: needs an ad-allocation problem (dlp_problem_create_adalloc)");
        return DLP_ERR_ARG;
    }
    if (o.binary && (o.intervals < 1 || o.intervals > dlp::mw::kBinMaxRatios)) {
        set_error("dlp_mw: binary mode needs 1 <= intervals <= 8");
        return DLP_ERR_ARG;
    }
    if (!(o.epsilon > 0.0 && o.epsilon < 1.0)) {
        set_error("dlp_mw: epsilon must be in (0, 1)");
        return DLP_ERR_ARG;
    }
    auto* m = new (std::nothrow) dlp_mw();
    if (!m) return DLP_ERR_OOM;
    int rc = DLP_OK;
    try {
        rc = mw_init(prob, &o, m);
    } catch (const std::exception& e) {
        set_error(std::string("dlp_mw_create: ") + e.what());
        rc = DLP_ERR_OOM;
    }
    if (rc != DLP_OK) {
        mw_free(m);
        return rc;
    }
    *out = m;
    return DLP_OK;
}

int dlp_mw_run(dlp_mw* m, int iterations, dlp_mw_iter* log, double* kernel_ms) {
    if (!m || iterations < 0) return DLP_ERR_ARG;
    MW_TRY(hipSetDevice(m->device));
    if (iterations > m->log_cap) {
        if (m->dlog) (void)hipFree(m->dlog);
        m->dlog = nullptr;
        MW_TRY(hipMalloc(&m->dlog, sizeof(dlp_mw_iter) * std::max(iterations, 1)));
        m->log_cap = iterations;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    MW_TRY(hipEventCreate(&e0));
    MW_TRY(hipEventCreate(&e1));
    MW_TRY(hipEventRecord(e0, m->stream));
    int rc = DLP_OK;
    for (int k = 0; k < iterations && rc == DLP_OK; ++k) rc = mw_iteration(m, m->dlog + k);
    if (rc == DLP_OK) {
        MW_TRY(hipEventRecord(e1, m->stream));
        MW_TRY(hipStreamSynchronize(m->stream));
        float ms = 0.f;
        MW_TRY(hipEventElapsedTime(&ms, e0, e1));
        if (kernel_ms) *kernel_ms = ms;
        if (log && iterations > 0)
            MW_TRY(hipMemcpy(log, m->dlog, sizeof(dlp_mw_iter) * iterations, hipMemcpyDeviceToHost));
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}

int dlp_mw_solution(dlp_mw* m, double* x_avg, double* x_current, double* weights) {
    if (!m) return DLP_ERR_ARG;
    MW_TRY(hipSetDevice(m->device));
    MW_TRY(hipStreamSynchronize(m->stream));
    std::vector<double> xi(m->nnz);
    if (x_avg) {
        MW_TRY(hipMemcpy(xi.data(), m->xa, sizeof(double) * m->nnz, hipMemcpyDeviceToHost));
        for (int64_t k = 0; k < m->nnz; ++k) x_avg[k] = xi[m->var_to_imp[k]];
    }
    if (x_current) {
        MW_TRY(hipMemcpy(xi.data(), m->x, sizeof(double) * m->nnz, hipMemcpyDeviceToHost));
        for (int64_t k = 0; k < m->nnz; ++k) x_current[k] = xi[m->var_to_imp[k]];
    }
    if (weights) MW_TRY(hipMemcpy(weights, m->w, sizeof(double) * m->A, hipMemcpyDeviceToHost));
    return DLP_OK;
}

void dlp_mw_free(dlp_mw* m) { mw_free(m); }

}  // extern "C"
