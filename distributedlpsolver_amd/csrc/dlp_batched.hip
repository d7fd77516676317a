// dlp_batched.hip — C5: thousands of independent small LPs, one workgroup per
// LP, the tableau's nonbasic columns + RHS resident in LDS ((m+1) x (n+1) fp64:
// 65 x 129 x 8 B = 67 KB at 64 x 128, two workgroups per CU of 160 KB; 34 KB at
// 64 x 64, four).  HBM is touched once per LP (load the generated tableau,
// store the outputs); every pivot is LDS traffic plus workgroup barriers
// (SURVEY.md §8a row a6).
//
// Pivot rule and arithmetic are exactly the big-tableau path's (dlp.h header):
// Dantzig/Bland pricing with index ties, ratio test with basis-index ties,
// IEEE division for the pivot row, fma elimination, colq == 0 rows untouched.
// Reference analog: the per-impression subproblems solved independently in
// GlobalProblem::ConstructPrimal, R/global_problem.cpp:270-274.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "dlp_host.h"
#include "dlp_internal.h"

namespace dlp {
namespace {

__device__ inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ inline uint64_t skey(uint64_t seed, uint64_t s) {
    return mix64(seed ^ (0x9E3779B97F4A7C15ULL * (s + 1)));
}
__device__ inline double u01(uint64_t key, uint64_t idx) {
    return (double)(mix64(key + idx) >> 11) * 0x1.0p-53;
}

// Tableaus of the batch in HBM: LP k at T + k*(m+1)*ld, generated with seed+k
// (same spec as generate_rows_kernel: one wave per row, strided fma chains +
// fixed halving tree for b).  blockIdx.y = LP, waves of blockIdx.x = rows.
__global__ __launch_bounds__(256) void batched_generate_kernel(double* __restrict__ T, int64_t ld,
                                                               int64_t m, int64_t n, int kind,
                                                               uint64_t seed) {
    const int lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t sk = seed + blockIdx.y;
    double* base = T + (int64_t)blockIdx.y * (m + 1) * ld;
    const int64_t N = n + m;
    if (i < m) {
        const uint64_t kA = skey(sk, 1), kX = skey(sk, 2), kU = skey(sk, 3), kD = skey(sk, 5);
        double* r = base + i * ld;
        // degenerate family: ~50% "cone" rows with A in [-1,1) and b = 0
        const bool cone = kind == DLP_GEN_DEGENERATE && (mix64(kD + (uint64_t)i) >> 63) == 0;
        double acc = 0.0;
        for (int64_t j = lane; j < n; j += 64) {
            const double u = u01(kA, (uint64_t)(i * n + j));
            const double a = cone ? 2.0 * u - 1.0 : u;
            r[j] = a;
            acc = __builtin_fma(a, u01(kX, (uint64_t)j), acc);
        }
#pragma unroll
        for (int w = 32; w >= 1; w >>= 1) acc = acc + __shfl_down(acc, w);
        double bi = __shfl(acc, 0) + u01(kU, (uint64_t)i);
        if (cone) bi = 0.0;
        for (int64_t j = n + lane; j < ld; j += 64) r[j] = (j == n + i) ? 1.0 : (j == N ? bi : 0.0);
    } else if (i == m) {
        double* z = base + m * ld;
        const uint64_t kC = skey(sk, 4);
        for (int64_t j = lane; j < ld; j += 64) z[j] = (j < n) ? -u01(kC, (uint64_t)j) : 0.0;
    }
}

struct BatchOut {
    double* objective;
    int32_t* status;
    int64_t* npivots;
    int32_t* basis;
    dlp_pivot* logs;
    int64_t log_cap;
    uint64_t* stamps;   // diagnostics (DLP_BATCH_STAMPS): LP 0's phase clocks, [64 pivots][8]
};

// One workgroup = one LP.  The LDS holds only the NONBASIC columns of the
// tableau (+ the RHS): a basic variable's column is a unit vector, so storing
// it buys nothing, and dropping it takes the 64 x 128 tableau from 100 KB to
// 67 KB (two LPs per CU instead of one) and 64 x 64 from 67 KB to 34 KB.
// LDS image: T[(m+1)][W] with W = n + 1 (slots 0..n-1, RHS at slot n),
// colq[m+1], prow[W], var[n] (the variable in each slot), basis[m], scratch.
//
// Same values as the full tableau: when q enters at slot s_q and l leaves row
// p, slot s_q takes l's column.  In the full tableau that column is e_p (1.0
// exactly at row p, a signed zero elsewhere), so its new entries are
// prow_l = 1.0 / piv at row p and fma(-colq[i], prow_l, 0) elsewhere (or the
// zero, when colq[i] == 0): the same bits as the full update, up to the sign
// of a zero, which reaches no output (every later value that depends on it is
// a fma / division whose result does not).  Pricing runs over the slots with
// the full tableau's order: min z, ties -> smallest VARIABLE index; Bland ->
// the smallest variable index with z < -tol.
__global__ __launch_bounds__(512) void batched_solve_kernel(const double* __restrict__ Tg,
                                                            int64_t ldg, int m, int n,
                                                            int64_t max_pivots, int pricing,
                                                            double tol_dj, double tol_piv,
                                                            BatchOut out) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int N = n + m, W = n + 1;
    double* T = smem;                                   // (m+1) x W
    double* colq = T + (m + 1) * W;                     // m+1
    double* prow = colq + (m + 1);                      // W
    int32_t* var = (int32_t*)(prow + W);                // n
    int32_t* basis = var + n;                           // m
    // scratch: [0] q (variable), [1] slot of q, [2] p, [3] status, [4] bland
    int32_t* sI = basis + m;
    double* sD = (double*)(sI + 6 + ((n + m) & 1));     // piv, ratio (8-B aligned)

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int64_t lp = blockIdx.x;
    const double* src = Tg + lp * (m + 1) * ldg;
    for (int i = 0; i <= m; ++i)
        for (int s = tid; s < W; s += blockDim.x) T[i * W + s] = src[(int64_t)i * ldg + (s < n ? s : N)];
    for (int s = tid; s < n; s += blockDim.x) var[s] = s;
    for (int i = tid; i < m; i += blockDim.x) basis[i] = n + i;
    if (tid == 0) {
        sI[3] = DLP_RUNNING;
        sI[4] = pricing == DLP_PRICING_BLAND ? 1 : 0;
    }
    __syncthreads();

    int64_t k = 0;
    for (; k < max_pivots; ++k) {
        // ---- a1 pricing (wave 0): lexicographic (z, variable) min + first variable < -tol
        if (wid == 0) {
            double zmin = __builtin_inf();
            int vmin = kNoIndex, smin = -1, vb = kNoIndex, sb = -1;
            const double* z = T + m * W;
            for (int s = lane; s < n; s += 64) {
                const double v = z[s];
                const int vr = var[s];
                if (v < zmin || (v == zmin && vr < vmin)) { zmin = v; vmin = vr; smin = s; }
                if (v < -tol_dj && vr < vb) { vb = vr; sb = s; }
            }
#pragma unroll
            for (int sh = 32; sh >= 1; sh >>= 1) {
                const double oz = __shfl_xor(zmin, sh);
                const int ov = __shfl_xor(vmin, sh), os = __shfl_xor(smin, sh);
                const int ob = __shfl_xor(vb, sh), osb = __shfl_xor(sb, sh);
                if (oz < zmin || (oz == zmin && ov < vmin)) { zmin = oz; vmin = ov; smin = os; }
                if (ob < vb) { vb = ob; sb = osb; }
            }
            if (lane == 0) {
                int q = kNoIndex, sq = -1;
                if (sI[4]) {
                    q = vb;
                    sq = sb;
                } else if (vmin != kNoIndex && zmin < -tol_dj) {
                    q = vmin;
                    sq = smin;
                }
                sI[0] = (q == kNoIndex) ? -1 : q;
                sI[1] = sq;
            }
        }
        __syncthreads();
        const int q = sI[0], sq = sI[1];
        if (q < 0) {
            if (tid == 0) sI[3] = DLP_OK;
            break;
        }
        // ---- a2 ratio test (wave 0) + colq capture (all)
        for (int i = tid; i <= m; i += blockDim.x) colq[i] = T[i * W + sq];
        if (wid == 0) {
            Cand best;
            best.valid = 0; best.ratio = 0.0; best.basis_var = kNoIndex; best.row = -1;
            best.pad0 = 0; best.pivot = 0.0;
            for (int i = lane; i < m; i += 64) {
                const double a = T[i * W + sq];
                if (a > tol_piv) {
                    double rhs = T[i * W + n];
                    if (!(rhs > 0.0)) rhs = 0.0;
                    Cand c;
                    c.ratio = rhs / a; c.basis_var = basis[i]; c.row = i; c.valid = 1;
                    c.pad0 = 0; c.pivot = a;
                    if (cand_better(c, best)) best = c;
                }
            }
#pragma unroll
            for (int sh = 32; sh >= 1; sh >>= 1) {
                Cand o;
                o.ratio = __shfl_xor(best.ratio, sh);
                o.basis_var = __shfl_xor(best.basis_var, sh);
                o.row = __shfl_xor(best.row, sh);
                o.valid = __shfl_xor(best.valid, sh);
                o.pad0 = 0;
                o.pivot = __shfl_xor(best.pivot, sh);
                if (cand_better(o, best)) best = o;
            }
            if (lane == 0) {
                if (!best.valid) {
                    sI[2] = -1;
                } else {   // a4 select + log
                    const int p = best.row;
                    const int leaving = basis[p];
                    basis[p] = q;
                    var[sq] = leaving;   // the entering slot now holds the leaving variable
                    sI[2] = p;
                    sI[4] = (pricing == DLP_PRICING_BLAND) ? 1 : (best.ratio == 0.0 ? 1 : 0);
                    sD[0] = best.pivot;
                    sD[1] = best.ratio;
                    if (out.logs && k < out.log_cap) {
                        dlp_pivot e;
                        e.q = q; e.p = p; e.leaving = leaving; e.pad = 0;
                        e.ratio = best.ratio; e.objective = 0.0;
                        out.logs[lp * out.log_cap + k] = e;
                    }
                }
            }
        }
        __syncthreads();
        const int p = sI[2];
        if (p < 0) {
            if (tid == 0) sI[3] = DLP_UNBOUNDED;
            break;
        }
        // ---- a3 pivot row (IEEE division), then the elimination: work items (slot,
        // row group), R row groups so that the lanes share it evenly; rows 8 at a time,
        // loads first
        const double piv = sD[0];
        for (int s = tid; s < W; s += blockDim.x) prow[s] = (s == sq ? 1.0 : T[p * W + s]) / piv;
        __syncthreads();
        {
            // R row groups with W * R <= blockDim.x: no lane takes a second item
            const int R = W >= (int)blockDim.x ? 1 : (int)(blockDim.x / W);
            const int rpg = (m + 1 + R - 1) / R;
            for (int item = tid; item < W * R; item += blockDim.x) {
                const int rg = item / W, s = item - rg * W;
                const bool ent = s == sq;               // slot of q -> column of the leaving var
                const double pj = prow[s];
                const int ib = rg * rpg, ie = min(ib + rpg, m + 1);
                for (int i0 = ib; i0 < ie; i0 += 8) {
                    double t[8], f[8];
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int i = min(i0 + u, ie - 1);
                        f[u] = colq[i];
                        t[u] = ent ? 0.0 : T[i * W + s];
                    }
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        const int i = i0 + u;
                        const double v = __builtin_fma(-f[u], pj, t[u]);
                        const double nv = (i == p) ? pj : (f[u] != 0.0 ? v : t[u]);
                        if (i < ie) T[i * W + s] = nv;
                    }
                }
            }
        }
        __syncthreads();
        if (tid == 0 && out.logs && k < out.log_cap)
            out.logs[lp * out.log_cap + k].objective = T[m * W + n];
    }
    if (tid == 0) {
        int stt = sI[3];
        if (stt == DLP_RUNNING) stt = DLP_PIVOT_LIMIT;
        if (out.status) out.status[lp] = stt;
        if (out.npivots) out.npivots[lp] = k;
        if (out.objective) out.objective[lp] = T[m * W + n];
    }
    if (out.basis)
        for (int i = tid; i < m; i += blockDim.x) out.basis[lp * m + i] = basis[i];
}

// C5, register-resident (round 3): at m = 64 one LANE owns one slot (column) of the
// nonbasic tableau, all 65 of its rows in 130 VGPRs (rows unrolled: no dynamic register
// index), so the elimination is 65 fmas per lane from registers with the column q read
// from LDS as a broadcast, and the pivot row is computed in place (each lane divides its
// own T[p][s]).  A workgroup of NW = ceil((n + 1) / 64) waves is one LP (192 lanes at
// 64 x 128, 129 of them owning a slot); no LDS holds the tableau, so 3 waves per SIMD fit:
// 4 LPs per CU at 64 x 128 (the LDS kernel: 2), 6 at 64 x 64 (4).  Per pivot: pricing
// (wave shuffles + one LDS partial per wave), the entering column written to LDS by its
// owner lane, the ratio test by wave 0 (one row per lane, which also keeps that row's RHS),
// 3 barriers.
// Same operations on the same values as batched_solve_kernel (same bits).
// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>): a register array indexed
// by I stays in registers (a #pragma unroll of 65 iterations may be left rolled, and the
// array then lives in scratch)
template <typename F, int... I>
__device__ __forceinline__ void each_(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void each(F&& f) {
    each_(f, std::make_integer_sequence<int, N>{});
}

// Wave-wide minimum by DPP (xor 1, xor 2, half-row and row mirrors, then the row broadcasts
// 15 and 31: the full minimum lands in lane 63, read back as a uniform value) — a few cycles
// per step against the LDS round trip of each ds_bpermute a shuffle costs.  No NaN reaches
// them (the callers map NaN to +inf first).
template <int CTRL, int RMASK>
__device__ __forceinline__ double dpp_f64(double v, double id) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v), d = __builtin_bit_cast(uint64_t, id);
    const uint32_t lo = __builtin_amdgcn_update_dpp((int)(uint32_t)d, (int)(uint32_t)u, CTRL, RMASK, 0xf, false);
    const uint32_t hi = __builtin_amdgcn_update_dpp((int)(uint32_t)(d >> 32), (int)(uint32_t)(u >> 32), CTRL, RMASK, 0xf, false);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double wave_min_f64(double v) {
    const double id = __builtin_inf();
    double o;
    o = dpp_f64<0xB1, 0xf>(v, id); v = o < v ? o : v;    // quad_perm [1,0,3,2]
    o = dpp_f64<0x4E, 0xf>(v, id); v = o < v ? o : v;    // quad_perm [2,3,0,1]
    o = dpp_f64<0x141, 0xf>(v, id); v = o < v ? o : v;   // row_half_mirror
    o = dpp_f64<0x140, 0xf>(v, id); v = o < v ? o : v;   // row_mirror
    o = dpp_f64<0x142, 0xa>(v, id); v = o < v ? o : v;   // row_bcast:15
    o = dpp_f64<0x143, 0xc>(v, id); v = o < v ? o : v;   // row_bcast:31
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, 63), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), 63);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
template <int CTRL, int RMASK>
__device__ __forceinline__ int dpp_i32(int v) {
    return __builtin_amdgcn_update_dpp(kNoIndex, v, CTRL, RMASK, 0xf, false);
}
// lane `l`'s value (l uniform, in an SGPR): two v_readlane_b32
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const uint64_t b = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)b, l), hi = __builtin_amdgcn_readlane((uint32_t)(b >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int wave_min_i32(int v) {
    v = min(v, dpp_i32<0xB1, 0xf>(v));
    v = min(v, dpp_i32<0x4E, 0xf>(v));
    v = min(v, dpp_i32<0x141, 0xf>(v));
    v = min(v, dpp_i32<0x140, 0xf>(v));
    v = min(v, dpp_i32<0x142, 0xa>(v));
    v = min(v, dpp_i32<0x143, 0xc>(v));
    return __builtin_amdgcn_readlane(v, 63);
}

// Rows of the register-resident elimination in inline asm.  The entering column's entry f
// and the pivot row index are the same for every lane of the LP, so each test is a uniform
// exec mask (all lanes or none) set by SALU, with no branch.  (hipcc, left to itself, turned the 2 x 65 tests into live vector masks
// and spilled them, or moved the register rows to scratch.)
// t := fma(-f, pj, t) unless f == +-0 (the eager rule leaves the row untouched).
// 8 rows, their masks from zm (bit r set: the entering column's row r is +-0, the row is skipped;
// the ratio test ballots it once per pivot), so a row costs two SALU instructions and its fma
// (round 5; rounds 3-4 compared every row on the VALU first, a VALU -> SALU dependency per row),
// with the entering column's entries taken from another lane's register by DPP:
// lane k of every 16-lane row holds entry 16 g + k (cq = colq[16 g + (lane & 15)], g = R0 / 16), and
// v_fmac_f64_dpp ... row_newbcast:k reads it for the whole row (neg modifier: fma(-f, pj, t), the
// eager operation), so the elimination waits for one LDS read per 16 rows instead of one per 8.
// cq is written only by an LDS load (no VALU write within two instructions of a DPP read:
// tests/test_isa.py); an SALU write of exec before a DPP op needs no wait state.
template <int R0>
__device__ __forceinline__ void elim8dpp(double* t, double cq, double pj, uint64_t zm) {
    uint64_t sv;
    // (a group with no +-0 entry, the common case on a dense LP, branches to the 8 fmas back to
    // back; the branch is inside the asm so the register allocator sees one block)
    asm volatile(
        "s_bfe_u64 %[sv], %[zm], %[bfe]\n\t"
        "s_cbranch_scc1 1f\n\t"
        "v_fmac_f64_dpp %[t0], -%[c], %[pj] row_newbcast:%[k0] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[t1], -%[c], %[pj] row_newbcast:%[k1] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[t2], -%[c], %[pj] row_newbcast:%[k2] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[t3], -%[c], %[pj] row_newbcast:%[k3] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[t4], -%[c], %[pj] row_newbcast:%[k4] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[t5], -%[c], %[pj] row_newbcast:%[k5] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[t6], -%[c], %[pj] row_newbcast:%[k6] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[t7], -%[c], %[pj] row_newbcast:%[k7] row_mask:0xf bank_mask:0xf\n\t"
        "s_branch 2f\n"
        "1:\n\t"
        "s_mov_b64 %[sv], exec\n\t"
        "s_bitcmp1_b64 %[zm], %[r0]\n\ts_cselect_b64 exec, 0, %[sv]\n\tv_fmac_f64_dpp %[t0], -%[c], %[pj] row_newbcast:%[k0] row_mask:0xf bank_mask:0xf\n\t"
        "s_bitcmp1_b64 %[zm], %[r1]\n\ts_cselect_b64 exec, 0, %[sv]\n\tv_fmac_f64_dpp %[t1], -%[c], %[pj] row_newbcast:%[k1] row_mask:0xf bank_mask:0xf\n\t"
        "s_bitcmp1_b64 %[zm], %[r2]\n\ts_cselect_b64 exec, 0, %[sv]\n\tv_fmac_f64_dpp %[t2], -%[c], %[pj] row_newbcast:%[k2] row_mask:0xf bank_mask:0xf\n\t"
        "s_bitcmp1_b64 %[zm], %[r3]\n\ts_cselect_b64 exec, 0, %[sv]\n\tv_fmac_f64_dpp %[t3], -%[c], %[pj] row_newbcast:%[k3] row_mask:0xf bank_mask:0xf\n\t"
        "s_bitcmp1_b64 %[zm], %[r4]\n\ts_cselect_b64 exec, 0, %[sv]\n\tv_fmac_f64_dpp %[t4], -%[c], %[pj] row_newbcast:%[k4] row_mask:0xf bank_mask:0xf\n\t"
        "s_bitcmp1_b64 %[zm], %[r5]\n\ts_cselect_b64 exec, 0, %[sv]\n\tv_fmac_f64_dpp %[t5], -%[c], %[pj] row_newbcast:%[k5] row_mask:0xf bank_mask:0xf\n\t"
        "s_bitcmp1_b64 %[zm], %[r6]\n\ts_cselect_b64 exec, 0, %[sv]\n\tv_fmac_f64_dpp %[t6], -%[c], %[pj] row_newbcast:%[k6] row_mask:0xf bank_mask:0xf\n\t"
        "s_bitcmp1_b64 %[zm], %[r7]\n\ts_cselect_b64 exec, 0, %[sv]\n\tv_fmac_f64_dpp %[t7], -%[c], %[pj] row_newbcast:%[k7] row_mask:0xf bank_mask:0xf\n\t"
        "s_mov_b64 exec, %[sv]\n"
        "2:"
        : [t0] "+v"(t[0]), [t1] "+v"(t[1]), [t2] "+v"(t[2]), [t3] "+v"(t[3]), [t4] "+v"(t[4]), [t5] "+v"(t[5]),
          [t6] "+v"(t[6]), [t7] "+v"(t[7]), [sv] "=&s"(sv)
        : [c] "v"(cq), [pj] "v"(pj), [zm] "s"(zm), [bfe] "n"(R0 | (8 << 16)), [r0] "n"(R0), [r1] "n"(R0 + 1), [r2] "n"(R0 + 2),
          [r3] "n"(R0 + 3), [r4] "n"(R0 + 4), [r5] "n"(R0 + 5), [r6] "n"(R0 + 6), [r7] "n"(R0 + 7),
          [k0] "n"(R0 % 16), [k1] "n"(R0 % 16 + 1), [k2] "n"(R0 % 16 + 2), [k3] "n"(R0 % 16 + 3),
          [k4] "n"(R0 % 16 + 4), [k5] "n"(R0 % 16 + 5), [k6] "n"(R0 % 16 + 6), [k7] "n"(R0 % 16 + 7)
        : "scc");
}
__device__ __forceinline__ void elim_row(double& t, double f, double pj) {
    uint64_t sv;
    asm volatile(
        "v_cmp_neq_f64_e32 vcc, 0, %[f]\n\t"
        "s_and_saveexec_b64 %[sv], vcc\n\t"
        "v_fma_f64 %[t], -%[f], %[pj], %[t]\n\t"
        "s_mov_b64 exec, %[sv]"
        : [t] "+v"(t), [sv] "=&s"(sv)
        : [f] "v"(f), [pj] "v"(pj)
        : "vcc");
}
// 8 rows at a time, one exec save/restore per block (exec is all lanes or none per row: p is
// uniform), so a row costs a compare, an exec select and one move.  tp := t[p]
template <int R0>
__device__ __forceinline__ void pick8(double& tp, const double* t, int p) {
    uint64_t sv;
    asm volatile("s_mov_b64 %[sv], exec\n\t"
                 "s_cmp_eq_u32 %[p], %[r0]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[d], %[t0]\n\t"
                 "s_cmp_eq_u32 %[p], %[r1]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[d], %[t1]\n\t"
                 "s_cmp_eq_u32 %[p], %[r2]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[d], %[t2]\n\t"
                 "s_cmp_eq_u32 %[p], %[r3]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[d], %[t3]\n\t"
                 "s_cmp_eq_u32 %[p], %[r4]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[d], %[t4]\n\t"
                 "s_cmp_eq_u32 %[p], %[r5]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[d], %[t5]\n\t"
                 "s_cmp_eq_u32 %[p], %[r6]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[d], %[t6]\n\t"
                 "s_cmp_eq_u32 %[p], %[r7]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[d], %[t7]\n\t"
                 "s_mov_b64 exec, %[sv]"
                 : [d] "+v"(tp), [sv] "=&s"(sv)
                 : [t0] "v"(t[0]), [t1] "v"(t[1]), [t2] "v"(t[2]), [t3] "v"(t[3]), [t4] "v"(t[4]),
                   [t5] "v"(t[5]), [t6] "v"(t[6]), [t7] "v"(t[7]), [p] "s"(p), [r0] "n"(R0), [r1] "n"(R0 + 1),
                   [r2] "n"(R0 + 2), [r3] "n"(R0 + 3), [r4] "n"(R0 + 4), [r5] "n"(R0 + 5), [r6] "n"(R0 + 6),
                   [r7] "n"(R0 + 7)
                 : "scc");
}
// t[R0 + k] := v where R0 + k == p
template <int R0>
__device__ __forceinline__ void set8(double* t, double v, int p) {
    uint64_t sv;
    asm volatile("s_mov_b64 %[sv], exec\n\t"
                 "s_cmp_eq_u32 %[p], %[r0]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[t0], %[v]\n\t"
                 "s_cmp_eq_u32 %[p], %[r1]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[t1], %[v]\n\t"
                 "s_cmp_eq_u32 %[p], %[r2]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[t2], %[v]\n\t"
                 "s_cmp_eq_u32 %[p], %[r3]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[t3], %[v]\n\t"
                 "s_cmp_eq_u32 %[p], %[r4]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[t4], %[v]\n\t"
                 "s_cmp_eq_u32 %[p], %[r5]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[t5], %[v]\n\t"
                 "s_cmp_eq_u32 %[p], %[r6]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[t6], %[v]\n\t"
                 "s_cmp_eq_u32 %[p], %[r7]\n\ts_cselect_b64 exec, %[sv], 0\n\tv_mov_b64 %[t7], %[v]\n\t"
                 "s_mov_b64 exec, %[sv]"
                 : [t0] "+v"(t[0]), [t1] "+v"(t[1]), [t2] "+v"(t[2]), [t3] "+v"(t[3]), [t4] "+v"(t[4]),
                   [t5] "+v"(t[5]), [t6] "+v"(t[6]), [t7] "+v"(t[7]), [sv] "=&s"(sv)
                 : [v] "v"(v), [p] "s"(p), [r0] "n"(R0), [r1] "n"(R0 + 1), [r2] "n"(R0 + 2), [r3] "n"(R0 + 3),
                   [r4] "n"(R0 + 4), [r5] "n"(R0 + 5), [r6] "n"(R0 + 6), [r7] "n"(R0 + 7)
                 : "scc");
}
// dst := src where ROW == p (p uniform)
template <int ROW>
__device__ __forceinline__ void move_if_row(double& dst, double src, int p) {
    uint64_t m, sv;
    asm volatile(
        "s_cmp_eq_u32 %[p], %[row]\n\t"
        "s_cselect_b64 %[m], -1, 0\n\t"
        "s_and_saveexec_b64 %[sv], %[m]\n\t"
        "v_mov_b64 %[d], %[s]\n\t"
        "s_mov_b64 exec, %[sv]"
        : [d] "+v"(dst), [m] "=&s"(m), [sv] "=&s"(sv)
        : [s] "v"(src), [p] "s"(p), [row] "n"(ROW)
        : "scc");
}
template <int M, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(3))) void batched_reg_kernel(const double* __restrict__ Tg, int64_t ldg, int n,
                                                           int64_t max_pivots, int pricing, double tol_dj,
                                                           double tol_piv, BatchOut out) {
    static_assert(M == 64, "one ratio-test row per lane of wave 0");
    constexpr int R = M + 1;   // rows, the objective row last
    __shared__ double s_colq[R];
    __shared__ double s_zv[NW];
    __shared__ int32_t s_zvar[NW], s_zslot[NW], s_bvar[NW], s_bslot[NW];
    __shared__ int32_t s_basis[M];
    __shared__ int32_t s_p, s_leave, s_bland;
    __shared__ double s_piv;
    __shared__ uint64_t s_zm;   // rows 0..63 of the entering column that are +-0 (the elimination's skip rule)
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int N = n + M;
    const int sl = tid;              // this lane's slot: < n a variable's column
    const bool own = sl < n;
    int var = sl < n ? sl : kNoIndex;   // the variable in the slot
    const int64_t lp = blockIdx.x;
    // buffer loads, one lane offset and the row in the scalar offset (a flat load per row
    // would hold 65 64-bit addresses in VGPRs next to the 65 values); lanes past the slots
    // read out of range, which returns +0
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Tg + lp * (int64_t)R * ldg), (short)0, (int)((int64_t)R * ldg * 8), 0x00020000);
    const int voff = own ? sl * 8 : 0x7fffff00;
    double t[R];
    each<R>([&](auto I) {
        t[I] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, (int)(I * ldg * 8), 0));
    });
    // wave 0, lane i keeps row i's RHS (the ratio test's) and every lane of wave 0 the objective
    // value T[M][N], each updated with the operations a column slot's elimination applies (same
    // bits): the RHS column needs no slot of its own, so n columns take ceil(n / 64) waves (round
    // 4: 64 x 128 in 2 waves instead of 3, 64 x 64 in 1 instead of 2; more LPs per CU)
    double rr = 0.0, zr = 0.0;
    if (wid == 0) {
        rr = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(((int64_t)lane * ldg + N) * 8), 0, 0));
        zr = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, (int)(((int64_t)M * ldg + N) * 8), 0, 0));
    }
    for (int i = tid; i < M; i += blockDim.x) s_basis[i] = n + i;
    if (tid == 0) s_bland = pricing == DLP_PRICING_BLAND ? 1 : 0;
    __syncthreads();
    int status = DLP_RUNNING;
    int64_t k = 0;
    auto stamp = [&](int ph) {
        if (out.stamps && lp == 0 && tid == 0 && k < 64) out.stamps[k * 8 + ph] = wall_clock64();
    };
    for (; k < max_pivots; ++k) {
        stamp(0);
        // ---- a1 pricing: lexicographic (z, variable) min; Bland: first variable with z < -tol.
        // Reduced field by field (min z, then the smallest variable among the lanes holding it;
        // the Bland variable apart): fewer cross-lane moves than shuffling the whole tuple.
        {
            const bool cand = sl < n;
            const double z = cand && t[M] < __builtin_inf() ? t[M] : __builtin_inf();   // (as z < zmin: NaN skipped)
            const double zmin = wave_min_f64(z);
            const int vz = cand && z == zmin ? var : kNoIndex;
            const int vbl = cand && z < -tol_dj ? var : kNoIndex;
            const int vmin = wave_min_i32(vz), vb = wave_min_i32(vbl);
            // the slots of the two winners (variables are distinct: one lane each)
            const uint64_t wz = __ballot(vz == vmin && vmin != kNoIndex);
            const uint64_t wb = __ballot(vbl == vb && vb != kNoIndex);
            if (lane == 0) {
                s_zv[wid] = zmin;
                s_zvar[wid] = vmin;
                s_zslot[wid] = wz ? wid * 64 + __ffsll((unsigned long long)wz) - 1 : -1;
                s_bvar[wid] = vb;
                s_bslot[wid] = wb ? wid * 64 + __ffsll((unsigned long long)wb) - 1 : -1;
            }
        }
        __syncthreads();
        stamp(1);
        int q = kNoIndex, sq = -1;
        {
            double zmin = s_zv[0];
            int vmin = s_zvar[0], smin = s_zslot[0], vb = s_bvar[0], sb = s_bslot[0];
#pragma unroll
            for (int w = 1; w < NW; ++w) {
                if (s_zv[w] < zmin || (s_zv[w] == zmin && s_zvar[w] < vmin)) {
                    zmin = s_zv[w]; vmin = s_zvar[w]; smin = s_zslot[w];
                }
                if (s_bvar[w] < vb) { vb = s_bvar[w]; sb = s_bslot[w]; }
            }
            if (s_bland) {
                q = vb; sq = sb;
            } else if (vmin != kNoIndex && zmin < -tol_dj) {
                q = vmin; sq = smin;
            }
        }
        if (q == kNoIndex) {
            status = DLP_OK;
            break;
        }
        // ---- the entering column to LDS (its owner lane)
        if (sl == sq) each<R>([&](auto I) { s_colq[I] = t[I]; });
        __syncthreads();
        stamp(2);
        // ---- a2 ratio test (wave 0, row = lane) + a4 select and log
        if (wid == 0) {
            // min ratio over the valid rows, then the smallest basis variable among the rows
            // holding it (cand_better's order), field by field
            const double a = s_colq[lane];
            const uint64_t zm = __ballot(a == 0.0);   // (-0 == 0: both skipped, as the eager rule)
            if (lane == 0) s_zm = zm;
            const bool valid = a > tol_piv;
            double ratio = __builtin_inf();
            if (valid) {
                double rhs = rr;
                if (!(rhs > 0.0)) rhs = 0.0;
                ratio = rhs / a;
            }
            const uint64_t anyv = __ballot(valid);
            const double rmin = wave_min_f64(ratio);
            const bool tie = valid && ratio == rmin;
            const int bv = s_basis[lane];
            const uint64_t ties = __ballot(tie);
            int wl = __ffsll((unsigned long long)ties) - 1;
            if (__popcll(ties) > 1) {   // exact ties: the smallest basis variable
                const int bmin = wave_min_i32(tie ? bv : kNoIndex);
                wl = __ffsll((unsigned long long)__ballot(tie && bv == bmin)) - 1;
            }
            Cand best;
            best.valid = anyv != 0 ? 1 : 0;
            best.row = wl;
            // (wl is uniform: v_readlane, no LDS round trip as __shfl's ds_bpermute)
            const int wls = __builtin_amdgcn_readfirstlane(wl < 0 ? 0 : wl);
            best.basis_var = anyv != 0 ? __builtin_amdgcn_readlane(bv, wls) : kNoIndex;
            best.ratio = anyv != 0 ? readlane_f64(ratio, wls) : 0.0;
            best.pivot = anyv != 0 ? readlane_f64(a, wls) : 0.0;
            best.pad0 = 0;
            if (lane == 0) {
                if (!best.valid) {
                    s_p = -1;
                } else {
                    const int p = best.row;
                    const int leaving = s_basis[p];
                    s_basis[p] = q;
                    s_leave = leaving;
                    s_p = p;
                    s_bland = (pricing == DLP_PRICING_BLAND) ? 1 : (best.ratio == 0.0 ? 1 : 0);
                    s_piv = best.pivot;
                    if (out.logs && k < out.log_cap) {
                        dlp_pivot e;
                        e.q = q; e.p = p; e.leaving = leaving; e.pad = 0;
                        e.ratio = best.ratio; e.objective = 0.0;
                        out.logs[lp * out.log_cap + k] = e;
                    }
                }
            }
        }
        __syncthreads();
        stamp(3);
        const int p = __builtin_amdgcn_readfirstlane(s_p);   // (uniform: an SGPR operand below)
        // the elimination's inputs, requested with p's (their LDS latency overlaps the pivot-row
        // division): the skip rule's row masks from the entering column's zero mask (SALU, no VALU
        // compare per row) and the entries for the DPP broadcast, 4 LDS reads per lane (elim8dpp)
        const uint64_t zm = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(s_zm >> 32)) << 32) |
                            __builtin_amdgcn_readfirstlane((uint32_t)s_zm);
        double cq[M / 16];
        each<M / 16>([&](auto G) { cq[G] = s_colq[16 * G + (lane & 15)]; });
        // (with them: the pivot, the objective row's entry and wave 0's row entry for its RHS update)
        const double piv = s_piv, fM = s_colq[M];
        const double fr = wid == 0 ? s_colq[lane] : 0.0;
        if (p < 0) {
            status = DLP_UNBOUNDED;
            break;
        }
        // ---- a3 pivot row (IEEE division, in place) and the elimination; the entering slot
        // takes the leaving variable's column (e_p before the pivot)
        const bool ent = sl == sq;
        if (ent) var = s_leave;
        double tp = 0.0;
        // tp = t[p]: only the group of 8 rows holding p (a uniform branch per group)
        each<M / 8>([&](auto G) { if ((p >> 3) == (int)G) pick8<8 * G>(tp, &t[8 * G], p); });
        move_if_row<M>(tp, t[M], p);
        const double pj = (ent ? 1.0 : tp) / piv;
        stamp(4);
        if (ent) each<R>([&](auto I) { t[I] = 0.0; });   // e_p before the pivot (see the LDS kernel)
        each<M / 8>([&](auto G) { elim8dpp<8 * G>(&t[8 * G], cq[G / 2], pj, zm); });
        elim_row(t[M], fM, pj);   // the objective row
        each<M / 8>([&](auto G) { if ((p >> 3) == (int)G) set8<8 * G>(&t[8 * G], pj, p); });   // row p := the pivot row
        move_if_row<M>(t[M], pj, p);
        if (wid == 0) {   // the RHS of row `lane` and the objective value, as a column slot updates its rows
            const double pjr = readlane_f64(rr, p) / piv;   // (p uniform)
            const double v = __builtin_fma(-fr, pjr, rr);
            rr = lane == p ? pjr : (fr != 0.0 ? v : rr);
            const double fz = fM;
            if (fz != 0.0) zr = __builtin_fma(-fz, pjr, zr);
        }
        stamp(5);
        if (tid == 0 && out.logs && k < out.log_cap) out.logs[lp * out.log_cap + k].objective = zr;
    }
    if (tid == 0) {
        int stt = status;
        if (stt == DLP_RUNNING) stt = DLP_PIVOT_LIMIT;
        if (out.status) out.status[lp] = stt;
        if (out.npivots) out.npivots[lp] = k;
        if (out.objective) out.objective[lp] = zr;
    }
    if (out.basis)
        for (int i = tid; i < M; i += blockDim.x) out.basis[lp * M + i] = s_basis[i];
}

}  // namespace
}  // namespace dlp

// A device's batch context, reused across dlp_batched_solve calls: the stream,
// the two timing events, the tableau buffer, one packed output buffer (objective | pivot count |
// status per LP, read back in ONE copy through a pinned staging buffer), basis and log buffers,
// each grown on demand and kept.  A fresh stream costs ~2 ms and the 7 allocations + frees ~1 ms
// on MI355X, more than the 64 x 128 batch's 0.8 ms kernel.  One context per device, taken for the
// whole call; a concurrent call on the same device builds and frees a private one as before.
// dlp_release_cached_memory frees them (dlp::batched_release).
namespace {
struct BatchCtx {
    int device = -1;
    hipStream_t s = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    void* dT = nullptr;   size_t capT = 0;
    void* dOut = nullptr; size_t capOut = 0;
    void* dB = nullptr;   size_t capB = 0;
    void* dL = nullptr;   size_t capL = 0;
    void* hOut = nullptr; size_t capH = 0;   // pinned
    void free_all() {
        if (device >= 0) (void)hipSetDevice(device);
        if (s) (void)hipStreamSynchronize(s);
        for (void* p : {dT, dOut, dB, dL})
            if (p) (void)hipFree(p);
        if (hOut) (void)hipHostFree(hOut);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (s) (void)hipStreamDestroy(s);
        (void)hipGetLastError();
        *this = BatchCtx{};
    }
};
constexpr int kBatchDevs = 64;
std::mutex g_batch_mu[kBatchDevs];
BatchCtx g_batch[kBatchDevs];

// grow *p to at least `bytes` (contents not kept)
hipError_t ensure_buf(void** p, size_t* cap, size_t bytes, bool pinned = false) {
    if (*cap >= bytes && *p) return hipSuccess;
    if (*p) (void)(pinned ? hipHostFree(*p) : hipFree(*p));
    *p = nullptr;
    *cap = 0;
    const hipError_t e = pinned ? hipHostMalloc(p, bytes, hipHostMallocDefault) : hipMalloc(p, bytes);
    if (e == hipSuccess) *cap = bytes;
    return e;
}

// restores the caller's current device on every return path
struct DeviceGuard {
    int dev = -1;
    DeviceGuard() { if (hipGetDevice(&dev) != hipSuccess) dev = -1; }
    ~DeviceGuard() { if (dev >= 0) (void)hipSetDevice(dev); }
};
}  // namespace

namespace dlp {
// Free the cached batch contexts of `device` (-1: all); returns the device bytes freed.
size_t batched_release(int device) {
    size_t n = 0;
    DeviceGuard g;
    for (int d = 0; d < kBatchDevs; ++d) {
        if (device >= 0 && d != device) continue;
        std::lock_guard<std::mutex> lk(g_batch_mu[d]);
        if (g_batch[d].device >= 0) {
            n += g_batch[d].capT + g_batch[d].capOut + g_batch[d].capB + g_batch[d].capL;
            g_batch[d].free_all();
        }
    }
    return n;
}
}  // namespace dlp

#define HIP_BTRY(expr)                                                               \
    do {                                                                             \
        hipError_t e_ = (expr);                                                      \
        if (e_ != hipSuccess) {                                                      \
            dlp::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));       \
            rc = DLP_ERR_HIP;                                                        \
            goto done;                                                               \
        }                                                                            \
    } while (0)

// The kernel dlp_batched_solve runs for an m x n batch, its lanes per LP and how many LPs one
// CU holds at once (the occupancy query with its VGPR / LDS footprint): C5's bound is per-pivot
// serial latency x this residency (bench.py --workload c5).
extern "C" int dlp_batched_occupancy(int64_t m, int64_t n, int device, int32_t* lps_per_cu,
                                     int32_t* threads_per_lp, int32_t* register_kernel) {
    if (m <= 0 || n <= 0) return DLP_ERR_ARG;
    const size_t lds = sizeof(double) * ((m + 1) * (n + 1) + (m + 1) + (n + 1)) + sizeof(int32_t) * (n + m + 8) +
                       sizeof(double) * 2 + 16;
    static const bool force_lds = std::getenv("DLP_BATCH_LDS") && std::atoi(std::getenv("DLP_BATCH_LDS")) == 1;
    const int nw = (int)((n + 63) / 64);
    const bool reg = !force_lds && m == 64 && nw >= 1 && nw <= 3;
    if (!reg && lds > 160 * 1024) return DLP_ERR_UNSUPPORTED;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        dlp::set_error("no HIP device visible (libdlp has no CPU fallback)");
        return DLP_ERR_NODEVICE;
    }
    DeviceGuard guard;   // the caller's current device is restored
    if (hipSetDevice(device) != hipSuccess) return DLP_ERR_HIP;
    int nb = 0, threads = 0;
    hipError_t e;
    if (reg) {
        threads = 64 * nw;
        e = nw == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, dlp::batched_reg_kernel<64, 1>, threads, 0)
          : nw == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, dlp::batched_reg_kernel<64, 2>, threads, 0)
                    : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, dlp::batched_reg_kernel<64, 3>, threads, 0);
    } else {
        threads = lds > 40 * 1024 ? 512 : 256;
        e = hipFuncSetAttribute((const void*)dlp::batched_solve_kernel,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e == hipSuccess)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, dlp::batched_solve_kernel, threads, lds);
    }
    if (e != hipSuccess) {
        dlp::set_error(std::string("dlp_batched_occupancy: ") + hipGetErrorString(e));
        return DLP_ERR_HIP;
    }
    if (lps_per_cu) *lps_per_cu = nb;
    if (threads_per_lp) *threads_per_lp = threads;
    if (register_kernel) *register_kernel = reg ? 1 : 0;
    return DLP_OK;
}

extern "C" int dlp_batched_solve(int kind, int64_t nlp, int64_t m, int64_t n, uint64_t seed,
                                 const dlp_options* opt, double* objective, int32_t* status,
                                 int64_t* npivots, int32_t* basis, dlp_pivot* logs,
                                 int64_t log_cap, double* kernel_ms) {
    dlp_options o;
    if (opt) o = *opt; else dlp_options_default(&o);
    if (nlp <= 0 || m <= 0 || n <= 0 || (kind != DLP_GEN_DENSE && kind != DLP_GEN_DEGENERATE) ||
        nlp > 65535 * 16 || log_cap < 0) {
        dlp::set_error("dlp_batched_solve: bad arguments");
        return DLP_ERR_ARG;
    }
    const int64_t N = n + m, ldg = (N + 1 + 15) / 16 * 16;
    const size_t lds = sizeof(double) * ((m + 1) * (n + 1) + (m + 1) + (n + 1)) + sizeof(int32_t) * (n + m + 8) +
                       sizeof(double) * 2 + 16;
    int rc = DLP_OK;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        dlp::set_error("no HIP device visible (libdlp has no CPU fallback)");
        return DLP_ERR_NODEVICE;
    }
    if (o.device < 0 || o.device >= ndev) {
        dlp::set_error("dlp_batched_solve: no such device");
        return DLP_ERR_ARG;
    }
    if (lds > 160 * 1024) {
        dlp::set_error("dlp_batched_solve: tableau does not fit in 160 KiB of LDS");
        return DLP_ERR_UNSUPPORTED;
    }
    DeviceGuard guard;
    BatchCtx priv;
    BatchCtx* c = &priv;
    std::unique_lock<std::mutex> lk;
    if (o.device < kBatchDevs) {
        lk = std::unique_lock<std::mutex>(g_batch_mu[o.device], std::try_to_lock);
        if (lk.owns_lock()) c = &g_batch[o.device];
    }
    uint64_t* dStamps = nullptr;
    dlp::BatchOut bo{};
    const size_t bOut = (sizeof(double) + sizeof(int64_t) + sizeof(int32_t)) * (size_t)nlp;
    double* dObj = nullptr;
    int64_t* dNp = nullptr;
    int32_t* dSt = nullptr;
    const bool want_log = logs && log_cap > 0;
    HIP_BTRY(hipSetDevice(o.device));
    c->device = o.device;
    if (!c->s) HIP_BTRY(hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking));
    if (!c->e0) HIP_BTRY(hipEventCreate(&c->e0));
    if (!c->e1) HIP_BTRY(hipEventCreate(&c->e1));
    HIP_BTRY(ensure_buf(&c->dT, &c->capT, sizeof(double) * nlp * (m + 1) * ldg));
    HIP_BTRY(ensure_buf(&c->dOut, &c->capOut, bOut));
    HIP_BTRY(ensure_buf(&c->hOut, &c->capH, bOut, true));
    if (basis) HIP_BTRY(ensure_buf(&c->dB, &c->capB, sizeof(int32_t) * nlp * m));
    if (want_log) HIP_BTRY(ensure_buf(&c->dL, &c->capL, sizeof(dlp_pivot) * nlp * log_cap));
    dObj = (double*)c->dOut;
    dNp = (int64_t*)(dObj + nlp);
    dSt = (int32_t*)(dNp + nlp);
    {
        hipStream_t s = c->s;
        double* dT = (double*)c->dT;
        dim3 gg((unsigned)((m + 1 + 3) / 4), (unsigned)nlp);
        dlp::batched_generate_kernel<<<gg, 256, 0, s>>>(dT, ldg, m, n, kind, seed);
        HIP_BTRY(hipGetLastError());
        bo.objective = dObj;
        bo.status = dSt;
        bo.npivots = dNp;
        bo.basis = basis ? (int32_t*)c->dB : nullptr;
        bo.logs = want_log ? (dlp_pivot*)c->dL : nullptr;
        bo.log_cap = want_log ? log_cap : 0;
        static const char* stamp_file = std::getenv("DLP_BATCH_STAMPS");
        if (stamp_file) {
            HIP_BTRY(hipMalloc(&dStamps, sizeof(uint64_t) * 64 * 8));
            HIP_BTRY(hipMemsetAsync(dStamps, 0, sizeof(uint64_t) * 64 * 8, s));
            bo.stamps = dStamps;
        }
        // m = 64 with n <= 192 columns: the register-resident kernel (DLP_BATCH_LDS=1: the LDS
        // kernel, for A/B); otherwise the LDS-resident one
        static const bool force_lds = std::getenv("DLP_BATCH_LDS") && std::atoi(std::getenv("DLP_BATCH_LDS")) == 1;
        const int nw = (int)((n + 63) / 64);
        const bool reg = !force_lds && m == 64 && nw >= 1 && nw <= 3;
        if (!reg)
            HIP_BTRY(hipFuncSetAttribute((const void*)dlp::batched_solve_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        HIP_BTRY(hipEventRecord(c->e0, s));
        if (reg) {
            if (nw == 1)
                dlp::batched_reg_kernel<64, 1><<<(unsigned)nlp, 64, 0, s>>>(dT, ldg, (int)n, o.max_pivots, o.pricing,
                                                                          o.tol_dj, o.tol_piv, bo);
            else if (nw == 2)
                dlp::batched_reg_kernel<64, 2><<<(unsigned)nlp, 128, 0, s>>>(dT, ldg, (int)n, o.max_pivots, o.pricing,
                                                                           o.tol_dj, o.tol_piv, bo);
            else
                dlp::batched_reg_kernel<64, 3><<<(unsigned)nlp, 192, 0, s>>>(dT, ldg, (int)n, o.max_pivots, o.pricing,
                                                                           o.tol_dj, o.tol_piv, bo);
        } else {
            // 512 lanes per LP when few LPs share a CU (LDS > 40 KB each), else 256
            const unsigned threads = lds > 40 * 1024 ? 512 : 256;
            dlp::batched_solve_kernel<<<(unsigned)nlp, threads, lds, s>>>(
                dT, ldg, (int)m, (int)n, o.max_pivots, o.pricing, o.tol_dj, o.tol_piv, bo);
        }
        HIP_BTRY(hipGetLastError());
        HIP_BTRY(hipEventRecord(c->e1, s));
        // read back only what the caller asked for: the packed outputs it wants in one copy
        // (objective | pivot counts | status are contiguous), basis and logs when requested
        const bool wo = objective != nullptr, wn = npivots != nullptr, ws = status != nullptr;
        if (wo || wn || ws) {
            const size_t from = wo ? 0 : wn ? sizeof(double) * nlp : (sizeof(double) + sizeof(int64_t)) * nlp;
            const size_t to = ws ? bOut : wn ? (sizeof(double) + sizeof(int64_t)) * nlp : sizeof(double) * nlp;
            HIP_BTRY(hipMemcpyAsync((char*)c->hOut + from, (char*)c->dOut + from, to - from,
                                    hipMemcpyDeviceToHost, s));
        }
        if (basis) HIP_BTRY(hipMemcpyAsync(basis, c->dB, sizeof(int32_t) * nlp * m, hipMemcpyDeviceToHost, s));
        if (want_log)
            HIP_BTRY(hipMemcpyAsync(logs, c->dL, sizeof(dlp_pivot) * nlp * log_cap, hipMemcpyDeviceToHost, s));
        HIP_BTRY(hipStreamSynchronize(s));
        if (kernel_ms) {
            float ms = 0.f;
            HIP_BTRY(hipEventElapsedTime(&ms, c->e0, c->e1));
            *kernel_ms = ms;
        }
        if (wo) std::memcpy(objective, c->hOut, sizeof(double) * nlp);
        if (wn) std::memcpy(npivots, (char*)c->hOut + sizeof(double) * nlp, sizeof(int64_t) * nlp);
        if (ws) std::memcpy(status, (char*)c->hOut + (sizeof(double) + sizeof(int64_t)) * nlp, sizeof(int32_t) * nlp);
        if (dStamps) {   // diagnostics only
            std::vector<uint64_t> h(64 * 8);
            HIP_BTRY(hipMemcpy(h.data(), dStamps, sizeof(uint64_t) * 64 * 8, hipMemcpyDeviceToHost));
            if (FILE* f = std::fopen(stamp_file, "wb")) {
                std::fwrite(h.data(), sizeof(uint64_t), h.size(), f);
                std::fclose(f);
            }
        }
    }
done:
    if (dStamps) (void)hipFree(dStamps);
    if (rc != DLP_OK || c == &priv) c->free_all();   // a failed context is rebuilt next call
    return rc;
}
