// dlp_kernels.hip — CDNA4 (gfx950) kernels of one simplex pivot on an
// HBM-resident fp64 tableau.  SURVEY.md §8a rows a1-a4.  The reference has no
// simplex; nearest reference analogs are cited per kernel.
//
// Per pivot, stream-ordered, no host round trip:
//   ratio_kernel    pricing reduce (q) + ratio test + colq capture + last-WG
//                   argmin (+ select when single rank)                [a1,a2,a4]
//   select_kernel   winner of the all-gathered rank candidates (nranks > 1) [a4]
//   prow_kernel     prow = T[p]/T[p][q] (owner) / INT64_MIN sentinel        [a3]
//   update_kernel   T -= colq (x) prow, streaming 16 B/lane, nt loads/stores,
//                   fused pricing partials of the next pivot             [a3,a1]
//
// Arithmetic is bit-for-bit the oracle's: explicit fma, IEEE division, argmins
// with exact compares and index tie-breaks (reduction-order independent).
// Built with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <cmath>

#include "dlp_internal.h"

namespace dlp {
namespace {

#include "dlp_device.h"

// ------------------------------------------------------------------ kernels

// a1 at start-up: pricing partials of the initial objective row, one per
// 512-column tile (the same tiling the update kernel's fused epilogue uses).
// cd.on (condensed tableau): the partials carry variable indices (var_of), as commit_row's
__global__ __launch_bounds__(kUpdThreads) void price_init_kernel(const double* __restrict__ zrow,
                                                                 int64_t nprice, int tile,
                                                                 PricePart* pp, double tol_dj, Cond cd) {
    __shared__ PricePart lds[4];
    PricePart acc = pp_empty();
    const int per_lane = tile / kUpdThreads;   // 2 or 4 columns per lane, ascending
    const int64_t j = (int64_t)blockIdx.x * tile + (int64_t)threadIdx.x * per_lane;
    for (int k = 0; k < per_lane; k += 2)
        if (j + k < nprice) {
            const double z0 = zrow[j + k];
            const double z1 = (j + k + 1 < nprice) ? zrow[j + k + 1] : 0.0;
            if (cd.on)
                price_pair_var(acc, z0, z1, cd.var_of[j + k], j + k + 1 < nprice ? cd.var_of[j + k + 1] : -1, tol_dj);
            else
                price_pair(acc, z0, z1, j + k, nprice, tol_dj);
        }
    acc = block_price(acc, lds);
    if (threadIdx.x == 0) pp[blockIdx.x] = acc;
}

// a1 + a2 (+ a4 when single rank).  Every workgroup re-derives q from the
// tile partials (<= a few KB, L2-resident) so no extra launch is needed; then
// one lane per local row (objective row included for colq) reads T[i][q] and
// T[i][N] (two strided 8-B loads), captures colq[i], and forms the ratio
// candidate.  The last workgroup to arrive (ticket; sc1 hand-off, no fences)
// reduces the per-WG partials.
// Nearest reference analog: the tolerance-gated tight-set test
// R/global_problem.cpp:372-380 and first-wins scans :335-361.
__global__ __launch_bounds__(kRatioThreads) void ratio_kernel(
    const double* __restrict__ T, int64_t ld, int64_t rows, int64_t rows_elig, int64_t ncols,
    int64_t row_first, const int32_t* basis, int32_t* basis_w, const PricePart* __restrict__ pp, int ntiles,
    DevState* st, double* __restrict__ colq, Cand* partials, Cand* cand_out, int nranks,
    double tol_dj, double tol_piv, int pricing, dlp_pivot* log, int64_t log_cap) {
    __shared__ PricePart lds_pp[4];
    __shared__ Cand lds_c[4];
    __shared__ int s_last;
    if (st->status != DLP_RUNNING) return;

    // ---- pricing: q from the column-tile partials
    PricePart acc = pp_empty();
    for (int k = threadIdx.x; k < ntiles; k += blockDim.x) pp_combine(acc, pp[k]);
    acc = block_price(acc, lds_pp);
    const int bland = st->bland;
    int32_t q;
    if (bland)
        q = acc.jbland;
    else
        q = (acc.jmin != kNoIndex && acc.zmin < -tol_dj) ? acc.jmin : kNoIndex;
    if (q == kNoIndex) {   // optimal: every WG agrees; WG 0 records it
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->q = -1;
            st->status = DLP_OK;
        }
        return;
    }

    // ---- ratio test over local rows
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    Cand c = cand_empty();
    if (i <= rows) {
        const double a = T[i * ld + q];
        colq[i] = a;
        if (i < rows_elig && a > tol_piv) {
            double rhs = T[i * ld + ncols];
            if (!(rhs > 0.0)) rhs = 0.0;
            c.ratio = rhs / a;
            c.row = (int32_t)(row_first + i);
            c.basis_var = basis[row_first + i];
            c.valid = 1;
            c.pivot = a;
        }
    }
    c = block_cand(c, lds_c);

    // ---- last-arriving workgroup reduces the partials.  No fences (an agent
    // release is an L2 write-back per workgroup on gfx950): write-through (sc1)
    // stores drained by vmcnt(0) before the ticket add, sc1 loads after it.
    typedef unsigned int u4v __attribute__((ext_vector_type(4)));
    constexpr int kAuxSc1 = 16;
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)partials, (short)0, (int)(gridDim.x * sizeof(Cand)), 0x00020000);
    if (threadIdx.x == 0) {
        const u4v* cv = (const u4v*)&c;
        __builtin_amdgcn_raw_buffer_store_b128(cv[0], prs, (int)(blockIdx.x * sizeof(Cand)), 0, kAuxSc1);
        __builtin_amdgcn_raw_buffer_store_b128(cv[1], prs, (int)(blockIdx.x * sizeof(Cand)) + 16, 0,
                                               kAuxSc1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev =
            __hip_atomic_fetch_add(&st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (prev == gridDim.x - 1);
    }
    __syncthreads();
    if (!s_last) return;
    Cand best = cand_empty();
    for (int k = threadIdx.x; k < (int)gridDim.x; k += blockDim.x) {
        Cand o;
        u4v* ov = (u4v*)&o;
        ov[0] = __builtin_amdgcn_raw_buffer_load_b128(prs, (int)(k * sizeof(Cand)), 0, kAuxSc1);
        ov[1] = __builtin_amdgcn_raw_buffer_load_b128(prs, (int)(k * sizeof(Cand)) + 16, 0, kAuxSc1);
        if (cand_better(o, best)) best = o;
    }
    best = block_cand(best, lds_c);
    if (threadIdx.x == 0) {
        st->ticket = 0;
        st->q = q;
        if (nranks == 1)
            do_select(st, best, q, basis_w, row_first, rows, pricing, log, log_cap);
        else
            cand_out[0] = best;
    }
}

// a4 for nranks > 1: every rank reduces the same all-gathered candidates in
// the same order, so all ranks agree on p with no MINLOC collective.
// Forced (Phase I drive-out) pivot: q travels in the candidate's pad0; a row
// with no usable column is redundant and the pivot is skipped.
__device__ inline void forced_select(DevState* st, const Cand& best, int32_t* basis,
                                     int64_t row_first, int64_t rows, int pricing,
                                     dlp_pivot* log, int64_t log_cap) {
    if (!best.valid) {
        st->status = kStatusSkip;
        return;
    }
    do_select(st, best, best.pad0, basis, row_first, rows, pricing, log, log_cap);
}

// Peer exchange (xp != NULL): the P candidates come from this rank's exchange block, each
// after its flag shows this exchange's seq (bounded wait; a stall -> kStatusXFail).
__global__ void select_kernel(const Cand* cands, int nranks, int32_t* basis, DevState* st,
                              int64_t row_first, int64_t rows, int pricing, dlp_pivot* log,
                              int64_t log_cap, int forced, int track, const XPeers* xp,
                              uint32_t seq, Cond cd) {
    __shared__ Cand s_c[kMaxRanks];
    __shared__ int s_ok;
    if (st->status != DLP_RUNNING) return;   // uniform: every rank holds the same status
    if (xp) {
        if (!x_gather_cands(xp, seq, s_c, &s_ok)) {
            if (threadIdx.x == 0) st->status = kStatusXFail;
            return;
        }
        cands = s_c;
    }
    if (threadIdx.x != 0) return;
    Cand best = cand_empty();
    for (int r = 0; r < nranks; ++r)
        if (cand_better(cands[r], best)) best = cands[r];
    if (forced)
        forced_select(st, best, basis, row_first, rows, pricing, log, log_cap);
    else
        do_select(st, best, st->q, basis, row_first, rows, pricing, log, log_cap, track != 0, true, cd);
}

// ---- peer exchange, stand-alone kernels (the eager and Phase I -> II paths; the deferred
// kernels push and wait inside their own launches)
__global__ void xcand_send_kernel(const XPeers* xp, uint32_t seq, const Cand* cand_send,
                                  const DevState* st) {
    if (st->status != DLP_RUNNING || threadIdx.x != 0) return;
    x_push_cand(xp, seq, cand_send[0]);
}

// Every rank's flag of candidate exchange seq (a barrier; the slots are not read).
__global__ void xwait_kernel(const XPeers* xp, uint32_t seq, DevState* st) {
    __shared__ Cand s_c[kMaxRanks];
    __shared__ int s_ok;
    if (st->status != DLP_RUNNING) return;
    if (!x_gather_cands(xp, seq, s_c, &s_ok) && threadIdx.x == 0) st->status = kStatusXFail;
}

// Owner: st->p_local >= 0 (a pivot row), or my_rank == owner_rank (owner_rank >= 0: the
// carried Phase II row, which travels while the status is "optimal" in phase 1).
__global__ __launch_bounds__(256) void xrow_send_kernel(const XPeers* xp, uint32_t seq,
                                                        const int64_t* __restrict__ bits, int64_t ld,
                                                        const DevState* st, int owner_rank,
                                                        int my_rank) {
    if (owner_rank < 0 && st->status != DLP_RUNNING) return;
    const bool owner = owner_rank >= 0 ? my_rank == owner_rank : st->p_local >= 0;
    if (!owner) return;   // uniform per launch
    const int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2;
    uint64_t v0 = 0, v1 = 0;
    if (j < ld) v0 = (uint64_t)bits[j];
    if (j + 1 < ld) v1 = (uint64_t)bits[j + 1];
    x_push_row_chunk(xp, seq, j, ld, v0, v1, (int)blockIdx.x);
}

__global__ __launch_bounds__(256) void xrow_recv_kernel(const XPeers* xp, uint32_t seq, int64_t ld,
                                                        int64_t* __restrict__ out, DevState* st,
                                                        int carry) {
    __shared__ int s_ok;
    if (!carry && st->status != DLP_RUNNING) return;
    if (threadIdx.x == 0) s_ok = x_wait(xp, x_rflag(xp, xp->me, blockIdx.x), seq) ? 1 : 0;
    __syncthreads();
    if (!s_ok) {
        if (threadIdx.x == 0) st->status = kStatusXFail;
        return;
    }
    const int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2;
    if (j < ld) {   // (ld is a multiple of 16: j + 1 < ld)
        uint64_t a = 0, b = 0;
        x_read_row_pair(xp, j, &a, &b);
        out[j] = (int64_t)a;
        out[j + 1] = (int64_t)b;
    }
}

// ---- general LPs: Phase I -> Phase II transition (include/dlp.h, "general LPs")
// Drive-out candidate for the artificial basic in global row `row`: the first
// priced column with |T[row][q]| > tol_piv (block min over each lane's first
// hit in its stride).  One workgroup; the owner rank produces the candidate.
__global__ __launch_bounds__(kRatioThreads) void drive_kernel(
    const double* __restrict__ T, int64_t ld, int64_t rows_elig, int64_t row_first, int64_t nprice,
    int64_t row, int32_t* basis, DevState* st, double tol_piv, Cand* cand_out, int nranks,
    int pricing, dlp_pivot* log, int64_t log_cap, int64_t rows) {
    __shared__ int32_t lds[kRatioThreads / 64];
    if (threadIdx.x == 0 && st->status == kStatusSkip) st->status = DLP_RUNNING;
    const int64_t pl = row - row_first;
    const bool mine = pl >= 0 && pl < rows_elig;
    int32_t q = kNoIndex;
    if (mine)
        for (int64_t j = threadIdx.x; j < nprice; j += blockDim.x)
            if (__builtin_fabs(T[pl * ld + j]) > tol_piv) {
                q = (int32_t)j;
                break;
            }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const int32_t o = __shfl_xor(q, m);
        q = o < q ? o : q;
    }
    if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = q;
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int w = 1; w < (int)(blockDim.x >> 6); ++w) q = lds[w] < q ? lds[w] : q;
    Cand c = cand_empty();
    if (mine && q != kNoIndex) {
        c.valid = 1;
        c.ratio = 0.0;
        c.row = (int32_t)row;
        c.basis_var = basis[row];
        c.pad0 = q;
        c.pivot = T[pl * ld + q];
    }
    if (nranks == 1) {
        if (st->status == DLP_RUNNING)
            forced_select(st, c, basis, row_first, rows, pricing, log, log_cap);
    } else {
        cand_out[0] = c;
    }
}

// colq capture for a forced pivot (q known only after the select).
__global__ void gather_q_kernel(const double* __restrict__ T, int64_t ld, int64_t rows,
                                const DevState* st, double* __restrict__ colq) {
    if (st->status != DLP_RUNNING) return;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= rows) colq[i] = T[i * ld + st->q];
}

// The carried Phase II objective row's fp64 bits (owner) / INT64_MIN (others),
// delivered to every rank by the same int64 MAX exchange as a pivot row.
__global__ __launch_bounds__(kProwThreads) void carry_out_kernel(const double* __restrict__ T,
                                                                 int64_t ld, int64_t carry_local,
                                                                 int64_t* __restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ld) return;
    if (carry_local >= 0) {
        const double v = T[carry_local * ld + j];
        out[j] = __builtin_bit_cast(int64_t, v);
    } else {
        out[j] = INT64_MIN;
    }
}

// Install the received row as the objective row; Phase II starts running.
__global__ __launch_bounds__(kProwThreads) void carry_in_kernel(double* __restrict__ T, int64_t ld,
                                                                int64_t rows,
                                                                const int64_t* __restrict__ in,
                                                                DevState* st, int pricing) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j < ld) T[rows * ld + j] = __builtin_bit_cast(double, in[j]);
    if (j == 0) {
        st->status = DLP_RUNNING;
        st->q = -1;
        st->bland = pricing == DLP_PRICING_BLAND ? 1 : 0;
    }
}

__global__ void set_status_kernel(DevState* st, int status) {
    if (threadIdx.x == 0) st->status = status;
}

// a3 (first half): normalised pivot row, IEEE division (never a reciprocal
// multiply).  Non-owner ranks write INT64_MIN, the identity of the int64 MAX
// all-reduce, which therefore delivers the owner's exact bits (signed zeros
// included) to every rank without a host-known broadcast root.
__global__ __launch_bounds__(kProwThreads) void prow_kernel(const double* __restrict__ T,
                                                            int64_t ld, const DevState* st,
                                                            int64_t* __restrict__ out) {
    if (st->status != DLP_RUNNING) return;
    const int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2;
    if (j >= ld) return;
    const int32_t pl = st->p_local;
    if (pl >= 0) {
        const double piv = st->piv;
        const d2 v = *(const d2*)(T + (int64_t)pl * ld + j);
        d2 r;
        r.x = v.x / piv;
        r.y = v.y / piv;
        *(d2*)(out + j) = r;
    } else {
        out[j] = INT64_MIN;
        out[j + 1] = INT64_MIN;
    }
}

template <bool NT>
__device__ inline d2 ld2(const double* p) {
    if constexpr (NT)
        return __builtin_nontemporal_load((const d2*)p);
    else
        return *(const d2*)p;
}
template <bool NT>
__device__ inline void st2(double* p, d2 v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, (d2*)p);
    else
        *(d2*)p = v;
}

// a3 (second half): the rank-1 elimination, the HBM-bound ~100% of a pivot.
// Workgroup (tile, band) owns columns [tile*TILE, +TILE) of rows
// [band*rb, +rb), TILE = 256 lanes x VEC doubles: each lane keeps its VEC prow
// values in registers for the whole band; colq[i] is wave-uniform (scalar
// load, or staged once per band in LDS when LDSQ); U rows are loaded before
// any is stored so every lane has U x VEC x 8 B in flight.  Rows with
// colq == 0 are skipped (no traffic); row p becomes prow.  The band holding
// the objective row also emits the next pivot's pricing partial for its tile
// and the objective value into the pivot log.
// Nearest reference analog: the 2x2 basis solve R/global_problem.cpp:393-405.
constexpr int kMaxBandLds = 256;

template <int VEC>
__device__ inline void price_lane(PricePart& acc, const d2* z, int64_t j, int64_t ncols,
                                  double tol_dj) {
#pragma unroll
    for (int v = 0; v < VEC / 2; ++v) price_pair(acc, z[v].x, z[v].y, j + 2 * v, ncols, tol_dj);
}

template <bool NT, int U, int VEC, bool LDSQ>
__global__ __launch_bounds__(kUpdThreads) void update_kernel(
    double* __restrict__ T, int64_t ld, int64_t rows, int64_t ncols, int64_t nprice,
    const double* __restrict__ colq, const double* __restrict__ prow, const DevState* st,
    PricePart* __restrict__ pp, int rb, double tol_dj, dlp_pivot* log, int64_t log_cap) {
    constexpr int TILE = kUpdThreads * VEC;
    constexpr int NV = VEC / 2;
    __shared__ PricePart lds_pp[4];
    __shared__ double lds_q[LDSQ ? kMaxBandLds + 16 : 1];
    if (st->status != DLP_RUNNING) return;
    const int tile = blockIdx.x;
    const int64_t j = (int64_t)tile * TILE + threadIdx.x * VEC;
    const int64_t width = (ncols + 16) & ~(int64_t)15;   // round16(N+1) <= ld: real columns
    const bool colok = j < width;   // ld % 16 == 0 and j % VEC == 0: the whole vector is in range
    // Lanes past ld (last, partial tile only) read a valid in-row address and
    // never store, so every load below is issued without a branch.
    const int64_t jc = colok ? j : width - VEC;
    d2 pr[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) pr[v] = *(const d2*)(prow + jc + 2 * v);
    const int64_t pl = st->p_local;
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;   // constraint rows only
    if constexpr (LDSQ) {
        for (int k = threadIdx.x; k < rb + U; k += blockDim.x)
            lds_q[k] = (i0 + k <= rows) ? colq[i0 + k] : 0.0;
        __syncthreads();
    }

    for (int64_t i = i0; i < iend; i += U) {
        d2 t[U][NV];
        double f[U];
        // All U loads in flight before the first use; a row that needs no
        // load (out of band, colq == 0, or the pivot row) reads the L2-hot
        // prow line instead of branching.
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t ii = i + u;
            if constexpr (LDSQ)
                f[u] = lds_q[ii - i0];
            else
                f[u] = colq[ii];   // colq is padded by kColqPad: always a valid read
            const bool need = (ii < iend) && (ii != pl) && (f[u] != 0.0);
            const double* src = need ? (T + ii * ld + jc) : (prow + jc);
#pragma unroll
            for (int v = 0; v < NV; ++v) t[u][v] = ld2<NT>(src + 2 * v);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t ii = i + u;
            if ((ii < iend) && (ii == pl || f[u] != 0.0)) {   // wave-uniform
#pragma unroll
                for (int v = 0; v < NV; ++v) {
                    d2 o;
                    o.x = __builtin_fma(-f[u], pr[v].x, t[u][v].x);
                    o.y = __builtin_fma(-f[u], pr[v].y, t[u][v].y);
                    if (ii == pl) o = pr[v];
                    if (colok) st2<NT>(T + ii * ld + j + 2 * v, o);
                }
            }
        }
    }

    if (i0 + rb > rows) {   // this band holds the objective row (local index `rows`)
        const double f = colq[rows];
        double* zp = T + rows * ld + jc;
        d2 z[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            z[v] = *(const d2*)(zp + 2 * v);
            if (f != 0.0 && colok) {
                z[v].x = __builtin_fma(-f, pr[v].x, z[v].x);
                z[v].y = __builtin_fma(-f, pr[v].y, z[v].y);
                *(d2*)(zp + 2 * v) = z[v];
            }
        }
        PricePart acc = pp_empty();
        if (colok) price_lane<VEC>(acc, z, j, nprice, tol_dj);
        acc = block_price(acc, lds_pp);
        if (threadIdx.x == 0) pp[tile] = acc;
        if (log && colok && j <= ncols && ncols < j + VEC) {
            const int64_t k = st->npivots - 1;
            const int64_t o = ncols - j;
            if (k >= 0 && k < log_cap) log[k].objective = (o & 1) ? z[o >> 1].y : z[o >> 1].x;
        }
    }
}

// Dense fast path of the same elimination.  The band's colq values are staged
// in LDS once; when no row of the band has colq == 0 and the pivot row is not
// in it (the common case on dense tableaus) every group of U rows is issued as
// U unconditional 16-B loads per lane from one uniform row pointer, then U
// fma pairs and U stores, with no per-row uniform state in scalar registers.
// Otherwise the band takes the general per-row path.  Results are identical
// to update_kernel (same fma per element, same skipped rows).
template <bool NT, int U, int THREADS>
__global__ __launch_bounds__(THREADS) void update_fast_kernel(
    double* __restrict__ T, int64_t ld, int64_t rows, int64_t ncols, int64_t nprice,
    const double* __restrict__ colq, const double* __restrict__ prow, const DevState* st,
    PricePart* __restrict__ pp, int rb, double tol_dj, dlp_pivot* log, int64_t log_cap) {
    constexpr int TILE = THREADS * 2;
    __shared__ PricePart lds_pp[THREADS / 64];
    __shared__ double lds_q[kMaxBandLds + 16];
    if (st->status != DLP_RUNNING) return;
    const int tile = blockIdx.x;
    const int64_t j = (int64_t)tile * TILE + threadIdx.x * 2;
    const int64_t width = (ncols + 16) & ~(int64_t)15;   // round16(N+1) <= ld: real columns
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - 2;
    const d2 pr = *(const d2*)(prow + jc);
    const int64_t pl = st->p_local;
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    int sparse = 0;
    for (int k = threadIdx.x; k < rb + U; k += THREADS) {
        const double f = (i0 + k <= rows) ? colq[i0 + k] : 0.0;
        lds_q[k] = f;
        if (i0 + k < iend && f == 0.0) sparse = 1;
    }
    sparse = __syncthreads_or(sparse) || (pl >= i0 && pl < iend);

    int64_t i = i0;
    if (!sparse) {
        for (; i + U <= iend; i += U) {
            double* rp = T + i * ld + jc;
            d2 t[U];
#pragma unroll
            for (int u = 0; u < U; ++u) t[u] = ld2<NT>(rp + u * ld);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double f = lds_q[i - i0 + u];
                d2 o;
                o.x = __builtin_fma(-f, pr.x, t[u].x);
                o.y = __builtin_fma(-f, pr.y, t[u].y);
                if (colok) st2<NT>(rp + u * ld, o);
            }
        }
    }
    for (; i < iend; ++i) {   // general path: remainder rows, or a sparse / pivot band
        const double f = lds_q[i - i0];
        if (i == pl) {
            if (colok) st2<NT>(T + i * ld + j, pr);
        } else if (f != 0.0) {
            const d2 t = ld2<NT>(T + i * ld + jc);
            d2 o;
            o.x = __builtin_fma(-f, pr.x, t.x);
            o.y = __builtin_fma(-f, pr.y, t.y);
            if (colok) st2<NT>(T + i * ld + j, o);
        }
    }

    if (i0 + rb > rows) {   // objective row: update + next pivot's pricing partial + log
        const double f = colq[rows];
        double* zp = T + rows * ld + jc;
        d2 z = *(const d2*)zp;
        if (f != 0.0 && colok) {
            z.x = __builtin_fma(-f, pr.x, z.x);
            z.y = __builtin_fma(-f, pr.y, z.y);
            *(d2*)zp = z;
        }
        PricePart acc = pp_empty();
        if (colok) price_pair(acc, z.x, z.y, j, nprice, tol_dj);
        acc = block_price(acc, lds_pp);
        if (threadIdx.x == 0) pp[tile] = acc;
        if (log && colok && j <= ncols && ncols < j + 2) {
            const int64_t k = st->npivots - 1;
            if (k >= 0 && k < log_cap) log[k].objective = (ncols == j) ? z.x : z.y;
        }
    }
}

// Row-serial form: every lane handles one row at a time (load -> fma -> store),
// so each wave has at most one 16-B load and one store in flight.  The number
// of resident workgroups per CU (and with it the requests in flight per CU)
// is capped by the launcher through a dynamic-LDS reservation: on this
// streaming pattern fewer outstanding requests per CU measured FASTER
// (tuning log).  Same arithmetic and skip rules as update_kernel.
template <bool NT, int VEC>
__global__ __launch_bounds__(kUpdThreads) void update_serial_kernel(
    double* __restrict__ T, int64_t ld, int64_t rows, int64_t ncols, int64_t nprice,
    const double* __restrict__ colq, const double* __restrict__ prow, const DevState* st,
    PricePart* __restrict__ pp, int rb, double tol_dj, dlp_pivot* log, int64_t log_cap) {
    constexpr int TILE = kUpdThreads * VEC;
    constexpr int NV = VEC / 2;
    __shared__ PricePart lds_pp[4];
    __shared__ double lds_q[kMaxBandLds + 16];
    if (st->status != DLP_RUNNING) return;
    const int tile = blockIdx.x;
    const int64_t j = (int64_t)tile * TILE + threadIdx.x * VEC;
    const int64_t width = (ncols + 16) & ~(int64_t)15;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - VEC;
    d2 pr[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) pr[v] = *(const d2*)(prow + jc + 2 * v);
    const int64_t pl = st->p_local;
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    for (int k = threadIdx.x; k < rb; k += kUpdThreads)
        lds_q[k] = (i0 + k <= rows) ? colq[i0 + k] : 0.0;
    __syncthreads();
    for (int64_t i = i0; i < iend; ++i) {
        const double f = lds_q[i - i0];
        if (i == pl) {
            if (colok)
#pragma unroll
                for (int v = 0; v < NV; ++v) st2<NT>(T + i * ld + j + 2 * v, pr[v]);
        } else if (f != 0.0) {
            d2 t[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) t[v] = ld2<NT>(T + i * ld + jc + 2 * v);
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                d2 o;
                o.x = __builtin_fma(-f, pr[v].x, t[v].x);
                o.y = __builtin_fma(-f, pr[v].y, t[v].y);
                if (colok) st2<NT>(T + i * ld + j + 2 * v, o);
            }
        }
    }

    if (i0 + rb > rows) {   // objective row: update + next pivot's pricing partial + log
        const double f = colq[rows];
        double* zp = T + rows * ld + jc;
        d2 z[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            z[v] = *(const d2*)(zp + 2 * v);
            if (f != 0.0 && colok) {
                z[v].x = __builtin_fma(-f, pr[v].x, z[v].x);
                z[v].y = __builtin_fma(-f, pr[v].y, z[v].y);
                *(d2*)(zp + 2 * v) = z[v];
            }
        }
        PricePart acc = pp_empty();
        if (colok) price_lane<VEC>(acc, z, j, nprice, tol_dj);
        acc = block_price(acc, lds_pp);
        if (threadIdx.x == 0) pp[tile] = acc;
        if (log && colok && j <= ncols && ncols < j + VEC) {
            const int64_t k = st->npivots - 1;
            const int64_t o = ncols - j;
            if (k >= 0 && k < log_cap) log[k].objective = (o & 1) ? z[o >> 1].y : z[o >> 1].x;
        }
    }
}

// Software-pipelined streaming form: each lane keeps DEPTH rows in flight
// and, in steady state, retires one row (fma + store) per new load, so reads
// and writes interleave at row granularity instead of in bursts of U.  Same
// arithmetic and skip rules as update_kernel.
template <bool NT, int DEPTH, int VEC>
__global__ __launch_bounds__(kUpdThreads) void update_stream_kernel(
    double* __restrict__ T, int64_t ld, int64_t rows, int64_t ncols, int64_t nprice,
    const double* __restrict__ colq, const double* __restrict__ prow, const DevState* st,
    PricePart* __restrict__ pp, int rb, double tol_dj, dlp_pivot* log, int64_t log_cap) {
    constexpr int TILE = kUpdThreads * VEC;
    constexpr int NV = VEC / 2;
    __shared__ PricePart lds_pp[4];
    __shared__ double lds_q[kMaxBandLds + 16];
    if (st->status != DLP_RUNNING) return;
    const int tile = blockIdx.x;
    const int64_t j = (int64_t)tile * TILE + threadIdx.x * VEC;
    const int64_t width = (ncols + 16) & ~(int64_t)15;   // round16(N+1) <= ld: real columns
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - VEC;
    d2 pr[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) pr[v] = *(const d2*)(prow + jc + 2 * v);
    const int64_t pl = st->p_local;
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    for (int k = threadIdx.x; k < rb + DEPTH; k += kUpdThreads)
        lds_q[k] = (i0 + k <= rows) ? colq[i0 + k] : 0.0;
    __syncthreads();

    auto src_of = [&](int64_t ii) -> const double* {
        const bool need = (ii < iend) && (ii != pl) && (lds_q[ii - i0] != 0.0);
        return need ? (T + ii * ld + jc) : (prow + jc);
    };
    d2 t[DEPTH][NV];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
        const double* sp = src_of(i0 + d);
#pragma unroll
        for (int v = 0; v < NV; ++v) t[d][v] = ld2<NT>(sp + 2 * v);
    }
    for (int64_t i = i0; i < iend; i += DEPTH) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) {
            const int64_t ii = i + d;
            const double f = lds_q[ii - i0];
            d2 o[NV];
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                o[v].x = __builtin_fma(-f, pr[v].x, t[d][v].x);
                o[v].y = __builtin_fma(-f, pr[v].y, t[d][v].y);
                if (ii == pl) o[v] = pr[v];
            }
            // refill this slot with row ii + DEPTH before storing row ii
            const double* sp = src_of(ii + DEPTH);
#pragma unroll
            for (int v = 0; v < NV; ++v) t[d][v] = ld2<NT>(sp + 2 * v);
            if ((ii < iend) && (ii == pl || f != 0.0) && colok) {
#pragma unroll
                for (int v = 0; v < NV; ++v) st2<NT>(T + ii * ld + j + 2 * v, o[v]);
            }
        }
    }

    if (i0 + rb > rows) {   // objective row: update + next pivot's pricing partial + log
        const double f = colq[rows];
        double* zp = T + rows * ld + jc;
        d2 z[NV];
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            z[v] = *(const d2*)(zp + 2 * v);
            if (f != 0.0 && colok) {
                z[v].x = __builtin_fma(-f, pr[v].x, z[v].x);
                z[v].y = __builtin_fma(-f, pr[v].y, z[v].y);
                *(d2*)(zp + 2 * v) = z[v];
            }
        }
        PricePart acc = pp_empty();
        if (colok) price_lane<VEC>(acc, z, j, nprice, tol_dj);
        acc = block_price(acc, lds_pp);
        if (threadIdx.x == 0) pp[tile] = acc;
        if (log && colok && j <= ncols && ncols < j + VEC) {
            const int64_t k = st->npivots - 1;
            const int64_t o = ncols - j;
            if (k >= 0 && k < log_cap) log[k].objective = (o & 1) ? z[o >> 1].y : z[o >> 1].x;
        }
    }
}

// -------------------------------------------------------------- generators
// SURVEY.md §8a row a7 (build spec; restated independently in oracle/oracle.cpp).
__device__ inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__device__ inline uint64_t stream_key(uint64_t seed, uint64_t s) {
    return mix64(seed ^ (0x9E3779B97F4A7C15ULL * (s + 1)));
}
__device__ inline double unit01(uint64_t key, uint64_t idx) {
    return (double)(mix64(key + idx) >> 11) * 0x1.0p-53;
}

// One wavefront per local row: lane l writes A[i][l + 64k] (coalesced) and
// accumulates the strided fma chain of b_i; the 64 chains are combined by the
// fixed halving tree (shfl_down 32..1) that the oracle restates.
// rhs: the RHS column (N; n for a condensed tableau, which stores no slack columns)
__global__ __launch_bounds__(256) void generate_rows_kernel(double* __restrict__ T, int64_t ld,
                                                            int64_t rows, int64_t row_first,
                                                            int64_t m, int64_t n, int kind,
                                                            uint64_t seed, int64_t rhs) {
    const int lane = threadIdx.x & 63;
    const int64_t il = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (il >= rows) return;
    const int64_t i = row_first + il;
    const int64_t N = n + m;
    const uint64_t kA = stream_key(seed, 1), kX = stream_key(seed, 2), kU = stream_key(seed, 3),
                   kD = stream_key(seed, 5);
    double* r = T + il * ld;
    // degenerate family: ~50% "cone" rows with A in [-1,1) (2u-1, exact) and b = 0
    const bool cone = kind == DLP_GEN_DEGENERATE && (mix64(kD + (uint64_t)i) >> 63) == 0;
    double acc = 0.0;
    for (int64_t j = lane; j < n; j += 64) {
        const double u = unit01(kA, (uint64_t)(i * n + j));
        const double a = cone ? 2.0 * u - 1.0 : u;
        r[j] = a;
        acc = __builtin_fma(a, unit01(kX, (uint64_t)j), acc);
    }
#pragma unroll
    for (int w = 32; w >= 1; w >>= 1) acc = acc + __shfl_down(acc, w);
    double bi = __shfl(acc, 0) + unit01(kU, (uint64_t)i);
    if (kind == DLP_GEN_DEGENERATE && (mix64(kD + (uint64_t)i) >> 63) == 0) bi = 0.0;
    // slack identity column, RHS and zero padding: each cell written by one lane
    for (int64_t j = n + lane; j < ld; j += 64) r[j] = (j == n + i && rhs == N) ? 1.0 : (j == rhs ? bi : 0.0);
}

__global__ __launch_bounds__(256) void generate_objective_kernel(double* __restrict__ z,
                                                                 int64_t ld, int64_t n,
                                                                 uint64_t seed) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= ld) return;
    z[j] = (j < n) ? -unit01(stream_key(seed, 4), (uint64_t)j) : 0.0;
}

__global__ void gather_column_kernel(const double* __restrict__ T, int64_t ld, int64_t nrows,
                                     int64_t col, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nrows) out[i] = T[i * ld + col];
}

}  // namespace

// --------------------------------------------------------------- launchers
int ratio_blocks(const Geometry& g) {
    return (int)((g.rows + 1 + kRatioThreads - 1) / kRatioThreads);
}

int update_tile(int variant) {
    if (variant == 14) return 512 * 2;
    const bool v4 = (variant >= 4 && variant <= 6) || variant == 10 || variant == 11 ||
                    variant == 19 || variant == 20 || variant == 27 || variant == 28;
    return kUpdThreads * (v4 ? 4 : 2);
}
int update_variants() { return 30; }

hipError_t launch_price_init(const Geometry& g, PricePart* pp, double tol_dj, int variant,
                             hipStream_t s) {
    const double* z = g.T + g.rows * g.ld;
    const int tile = update_tile(variant);
    const int ntiles = (int)((g.width + tile - 1) / tile);
    price_init_kernel<<<ntiles, kUpdThreads, 0, s>>>(z, g.nprice, tile, pp, tol_dj, g.cd);
    return hipGetLastError();
}

hipError_t launch_ratio(const Geometry& g, const int32_t* basis_in, int32_t* basis_out,
                        const PricePart* pp, DevState* st, double* colq, Cand* partials,
                        int nblocks, Cand* cand_out, int nranks, double tol_dj, double tol_piv,
                        int pricing, dlp_pivot* log, int64_t log_cap, hipStream_t s) {
    ratio_kernel<<<nblocks, kRatioThreads, 0, s>>>(g.T, g.ld, g.rows, g.rows_elig, g.ncols,
                                                   g.row_first,
                                                   basis_in, basis_out, pp, g.ntiles, st, colq,
                                                   partials, cand_out, nranks, tol_dj, tol_piv,
                                                   pricing, log, log_cap);
    return hipGetLastError();
}

hipError_t launch_select(const Geometry& g, const Cand* cands, int nranks, int32_t* basis,
                         DevState* st, int pricing, dlp_pivot* log, int64_t log_cap,
                         hipStream_t s, bool forced, bool track, const XPeers* xp, uint32_t seq) {
    if (nranks > kMaxRanks) return hipErrorInvalidValue;
    select_kernel<<<1, 64, 0, s>>>(cands, nranks, basis, st, g.row_first, g.rows, pricing, log,
                                   log_cap, forced ? 1 : 0, track ? 1 : 0, xp, seq, g.cd);
    return hipGetLastError();
}

// Condensed tableau: slots [0, n) hold variables 0..n-1 (the structural columns), the RHS slot and
// the padding no variable; the slacks n..N-1 start basic; no slot has restarted.
__global__ void cond_init_kernel(Cond cd, int64_t n, int64_t N, int64_t ld, DevState* st) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < N) cd.slot_of[k] = k < n ? (int32_t)k : -1;
    if (k < ld) {
        cd.var_of[k] = k < n ? (int32_t)k : -1;
        cd.rst[k] = -1;
    }
    if (k == 0) {
        st->sq = -1;
        st->bser = 0;
        st->seal[0].ser = st->seal[1].ser = -1;
    }
}

hipError_t launch_cond_init(const Geometry& g, int64_t N, DevState* st, hipStream_t s) {
    if (!g.cd.on) return hipSuccess;
    const int64_t tot = N > g.ld ? N : g.ld;
    cond_init_kernel<<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(g.cd, g.ncols, N, g.ld, st);
    return hipGetLastError();
}

size_t xblock_layout(int nranks, int64_t ld, int nslot, XPeers* xp) {
    const int64_t P = nranks, S = nslot;
    const int64_t nch = (ld + kXChunk - 1) / kXChunk;
    const int64_t off_cslot = (2 * P * S + 7) / 8 * 8;
    const int64_t off_rflag = off_cslot + 8 * P * S;
    const int64_t off_row = (off_rflag + nch + 511) / 512 * 512;   // 4 KiB aligned
    if (xp) {
        xp->nranks = nranks;
        xp->nslot = nslot;
        xp->nchunks = nch;
        xp->off_cslot = off_cslot;
        xp->off_rflag = off_rflag;
        xp->off_row = off_row;
    }
    return (size_t)(off_row + (ld + kXChunk - 1) / kXChunk * kXChunk) * sizeof(uint64_t);
}

hipError_t launch_xcand_send(const XPeers* xp, uint32_t seq, const Cand* cand_send, const DevState* st,
                             hipStream_t s) {
    xcand_send_kernel<<<1, 64, 0, s>>>(xp, seq, cand_send, st);
    return hipGetLastError();
}

hipError_t launch_xwait(const XPeers* xp, uint32_t seq, DevState* st, hipStream_t s) {
    xwait_kernel<<<1, 64, 0, s>>>(xp, seq, st);
    return hipGetLastError();
}

hipError_t launch_xrow_send(const XPeers* xp, uint32_t seq, const int64_t* bits, int64_t ld,
                            const DevState* st, int owner_rank, int my_rank, hipStream_t s) {
    const int blocks = (int)((ld + kXChunk - 1) / kXChunk);
    xrow_send_kernel<<<blocks, 256, 0, s>>>(xp, seq, bits, ld, st, owner_rank, my_rank);
    return hipGetLastError();
}

hipError_t launch_xrow_recv(const XPeers* xp, uint32_t seq, int64_t ld, int64_t* out, DevState* st,
                            hipStream_t s) {
    const int blocks = (int)((ld + kXChunk - 1) / kXChunk);
    xrow_recv_kernel<<<blocks, 256, 0, s>>>(xp, seq, ld, out, st, 0);
    return hipGetLastError();
}

hipError_t launch_drive(const Geometry& g, int64_t row, int32_t* basis, DevState* st,
                        double tol_piv, Cand* cand_out, int nranks, int pricing, dlp_pivot* log,
                        int64_t log_cap, double* colq, hipStream_t s) {
    drive_kernel<<<1, kRatioThreads, 0, s>>>(g.T, g.ld, g.rows_elig, g.row_first, g.nprice, row,
                                             basis, st, tol_piv, cand_out, nranks, pricing, log,
                                             log_cap, g.rows);
    if (nranks == 1) return launch_gather_q(g, st, colq, s);
    return hipGetLastError();
}

hipError_t launch_gather_q(const Geometry& g, const DevState* st, double* colq, hipStream_t s) {
    const int64_t blocks = (g.rows + 1 + 255) / 256;
    gather_q_kernel<<<(unsigned)blocks, 256, 0, s>>>(g.T, g.ld, g.rows, st, colq);
    return hipGetLastError();
}

hipError_t launch_carry_out(const Geometry& g, int64_t carry_local, int64_t* out, hipStream_t s) {
    const int blocks = (int)((g.ld + kProwThreads - 1) / kProwThreads);
    carry_out_kernel<<<blocks, kProwThreads, 0, s>>>(g.T, g.ld, carry_local, out);
    return hipGetLastError();
}

hipError_t launch_carry_in(const Geometry& g, const int64_t* in, DevState* st, int pricing,
                           hipStream_t s) {
    const int blocks = (int)((g.ld + kProwThreads - 1) / kProwThreads);
    carry_in_kernel<<<blocks, kProwThreads, 0, s>>>(g.T, g.ld, g.rows, in, st, pricing);
    return hipGetLastError();
}

hipError_t launch_set_status(DevState* st, int status, hipStream_t s) {
    set_status_kernel<<<1, 64, 0, s>>>(st, status);
    return hipGetLastError();
}

hipError_t launch_prow(const Geometry& g, const DevState* st, int64_t* prow_bits, int nranks,
                       hipStream_t s) {
    (void)nranks;
    const int64_t pairs = g.ld / 2;
    const int blocks = (int)((pairs + kProwThreads - 1) / kProwThreads);
    prow_kernel<<<blocks, kProwThreads, 0, s>>>(g.T, g.ld, st, prow_bits);
    return hipGetLastError();
}

template <bool NT, int U, int VEC, bool LDSQ>
static void upd(const Geometry& g, const double* colq, const double* prow, const DevState* st,
                PricePart* pp, double tol_dj, dlp_pivot* log, int64_t log_cap, hipStream_t s) {
    constexpr int TILE = kUpdThreads * VEC;
    const int ntiles = (int)((g.width + TILE - 1) / TILE);
    const int64_t bands = (g.rows + 1 + g.rows_per_block - 1) / g.rows_per_block;
    dim3 grid(ntiles, (unsigned)bands);
    update_kernel<NT, U, VEC, LDSQ><<<grid, kUpdThreads, 0, s>>>(
        g.T, g.ld, g.rows, g.ncols, g.nprice, colq, prow, st, pp, g.rows_per_block, tol_dj,
        log, log_cap);
}

template <bool NT, int U, int THREADS>
static void updf(const Geometry& g, const double* colq, const double* prow, const DevState* st,
                 PricePart* pp, double tol_dj, dlp_pivot* log, int64_t log_cap, hipStream_t s) {
    constexpr int TILE = THREADS * 2;
    const int ntiles = (int)((g.width + TILE - 1) / TILE);
    const int64_t bands = (g.rows + 1 + g.rows_per_block - 1) / g.rows_per_block;
    dim3 grid(ntiles, (unsigned)bands);
    update_fast_kernel<NT, U, THREADS><<<grid, THREADS, 0, s>>>(
        g.T, g.ld, g.rows, g.ncols, g.nprice, colq, prow, st, pp, g.rows_per_block, tol_dj,
        log, log_cap);
}

template <bool NT, int DEPTH, int VEC>
static void upds(const Geometry& g, const double* colq, const double* prow, const DevState* st,
                 PricePart* pp, double tol_dj, dlp_pivot* log, int64_t log_cap, hipStream_t s) {
    constexpr int TILE = kUpdThreads * VEC;
    const int ntiles = (int)((g.width + TILE - 1) / TILE);
    const int64_t bands = (g.rows + 1 + g.rows_per_block - 1) / g.rows_per_block;
    dim3 grid(ntiles, (unsigned)bands);
    update_stream_kernel<NT, DEPTH, VEC><<<grid, kUpdThreads, 0, s>>>(
        g.T, g.ld, g.rows, g.ncols, g.nprice, colq, prow, st, pp, g.rows_per_block, tol_dj,
        log, log_cap);
}

// OCC = workgroups per CU allowed by a dynamic-LDS reservation (0 = no cap).
template <bool NT, int VEC, int OCC>
static void updr(const Geometry& g, const double* colq, const double* prow, const DevState* st,
                 PricePart* pp, double tol_dj, dlp_pivot* log, int64_t log_cap, hipStream_t s) {
    constexpr int TILE = kUpdThreads * VEC;
    const int ntiles = (int)((g.width + TILE - 1) / TILE);
    const int64_t bands = (g.rows + 1 + g.rows_per_block - 1) / g.rows_per_block;
    dim3 grid(ntiles, (unsigned)bands);
    // static LDS is ~2.2 KB; reserve the rest so that only OCC workgroups fit in 160 KiB
    const size_t dyn = OCC > 0 ? (size_t)(160 * 1024 / OCC) - 4096 : 0;
    update_serial_kernel<NT, VEC><<<grid, kUpdThreads, dyn, s>>>(
        g.T, g.ld, g.rows, g.ncols, g.nprice, colq, prow, st, pp, g.rows_per_block, tol_dj,
        log, log_cap);
}

template <bool NT>
static void upd_variant(int variant, const Geometry& g, const double* colq, const double* prow,
                        const DevState* st, PricePart* pp, double tol_dj, dlp_pivot* log,
                        int64_t log_cap, hipStream_t s) {
    switch (variant) {
        default:
        case 0: upd<NT, 4, 2, false>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 1: upd<NT, 8, 2, false>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 2: upd<NT, 4, 2, true>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 3: upd<NT, 8, 2, true>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 4: upd<NT, 4, 4, false>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 5: upd<NT, 2, 4, false>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 6: upd<NT, 4, 4, true>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 7: upd<NT, 16, 2, true>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 8: upd<NT, 16, 2, false>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 9: upd<NT, 32, 2, true>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 10: upd<NT, 8, 4, true>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 11: upd<NT, 16, 4, true>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 12: updf<NT, 16, 256>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 13: updf<NT, 8, 256>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 14: updf<NT, 16, 512>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 15: updf<NT, 32, 256>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 16: upds<NT, 1, 2>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 17: upds<NT, 2, 2>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 18: upds<NT, 4, 2>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 19: upds<NT, 1, 4>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 20: upds<NT, 2, 4>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 21: upds<NT, 8, 2>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 22: updr<NT, 2, 4>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 23: updr<NT, 2, 2>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 24: updr<NT, 2, 3>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 25: updr<NT, 2, 6>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 26: updr<NT, 2, 0>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 27: updr<NT, 4, 4>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 28: updr<NT, 4, 2>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
        case 29: updr<NT, 2, 5>(g, colq, prow, st, pp, tol_dj, log, log_cap, s); break;
    }
}

hipError_t launch_update(const Geometry& g, const double* colq, const double* prow,
                         const DevState* st, PricePart* pp, double tol_dj, dlp_pivot* log,
                         int64_t log_cap, bool nontemporal, int variant, hipStream_t s) {
    if (nontemporal)
        upd_variant<true>(variant, g, colq, prow, st, pp, tol_dj, log, log_cap, s);
    else
        upd_variant<false>(variant, g, colq, prow, st, pp, tol_dj, log, log_cap, s);
    return hipGetLastError();
}

hipError_t launch_generate(const Geometry& g, int kind, int64_t m, int64_t n, uint64_t seed,
                           hipStream_t s) {
    if (g.rows > 0) {
        const int wpb = 4;   // wavefronts (rows) per workgroup
        const int64_t blocks = (g.rows + wpb - 1) / wpb;
        generate_rows_kernel<<<(unsigned)blocks, 64 * wpb, 0, s>>>(g.T, g.ld, g.rows,
                                                                   g.row_first, m, n, kind, seed,
                                                                   g.cd.on ? n : n + m);
    }
    const int64_t zb = (g.ld + 255) / 256;
    generate_objective_kernel<<<(unsigned)zb, 256, 0, s>>>(g.T + g.rows * g.ld, g.ld, n, seed);
    return hipGetLastError();
}

hipError_t launch_gather_column(const double* T, int64_t ld, int64_t nrows, int64_t col,
                                double* out, hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    const int64_t blocks = (nrows + 255) / 256;
    gather_column_kernel<<<(unsigned)blocks, 256, 0, s>>>(T, ld, nrows, col, out);
    return hipGetLastError();
}

}  // namespace dlp
