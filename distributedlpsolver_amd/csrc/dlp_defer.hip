// dlp_defer.hip — deferred rank-k form of the pivot,
// gfx950.  Up to K pivots are chosen against the stale HBM tableau T0, then
// one pass applies them all: the tableau is streamed once per K pivots instead
// of once per pivot, and every value stays bit-identical to K eager rank-1
// updates (dlp_kernels.hip), because each element sees the same operations in
// the same order:
//   step l on row i:  i == p_l       -> T[i][c] := P[l][c]          (row p := prow)
//                     C[l][i] != 0   -> T[i][c] := fma(-C[l][i], P[l][c], T[i][c])
//                     C[l][i] == 0   -> untouched
// where C[l][i] = T_l[i][q_l] (row i's entry in the entering column just
// before step l) and P[l] = T_l[p_l] / T_l[p_l][q_l].  Per pivot only three
// things are needed from the current tableau, each re-derived by replaying
// the block's earlier steps on T0: column q (ratio_defer_kernel, one lane per
// row), the pivot row p (prow_defer_kernel) and the RHS column (kept current
// in `rhs`, one step per pivot).  The objective row is kept current in place
// (updated by the pivot-row kernel, which also emits the next pricing
// partials), and the pass (pass_kernel) skips it.
//
// Nearest reference analogs as for the eager kernels: the tight-set test
// R/global_problem.cpp:372-380 (ratio), first-wins scans :335-361 (pricing),
// the 2x2 basis solve :393-405 (elimination).  Built with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <utility>

#include "dlp_internal.h"

namespace dlp {
namespace {

#include "dlp_device.h"

typedef unsigned int u4v __attribute__((ext_vector_type(4)));
typedef unsigned int u2v __attribute__((ext_vector_type(2)));
// A double's bits as the b64 buffer-store operand, built from scalars: hipcc miscompiles a
// __builtin_bit_cast of an element of an ext_vector value (tests/test_isa.py source guard).
__device__ __forceinline__ u2v dbits(double v) {
    uint64_t u;
    __builtin_memcpy(&u, &v, sizeof(u));
    u2v w;
    w.x = (unsigned)u;
    w.y = (unsigned)(u >> 32);
    return w;
}

template <bool NT>
__device__ inline d2 ldv(const double* p) {
    if constexpr (NT)
        return __builtin_nontemporal_load((const d2*)p);
    else
        return *(const d2*)p;
}
template <bool NT>
__device__ inline double ldv1(const double* p) {
    if constexpr (NT)
        return __builtin_nontemporal_load(p);
    else
        return *p;
}
template <bool NT>
__device__ inline void stv1(double* p, double v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}
template <bool NT>
__device__ inline void stv(double* p, d2 v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, (d2*)p);
    else
        *(d2*)p = v;
}

// 16-B LDS-DMA (global_load_lds_dwordx4: lane x's 16 bytes land at the wave-uniform LDS
// address m0 + 16 x) issued from inline asm, so that hipcc does not count it: with the
// builtin it waits vmcnt(0) before the next LDS read or ordinary-load use, draining every
// DMA in flight (cdna_hip_programming.md, glds).  The callers retire their DMAs with counted
// waits of their own (vmwait), which hold because between two of them they issue no other
// vector-memory instruction, or a fixed number of them.  The lgkmcnt(0) orders the DMA's
// LDS write after this wave's earlier LDS reads of the slot it refills.
__device__ __forceinline__ void glds16(const void* g, uint32_t m0) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}
template <int N>
__device__ __forceinline__ void vmwait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p);
}

// a1 + a2 (+ a4 single rank) on the replayed column q.  Pricing as in the
// eager ratio_kernel.  Lane i: a = T_j[i][q] by replaying steps 0..j-1 on
// T0[i][q]; C[j][i] = a; the RHS cache advances by step j-1 (or is read from
// T0 when the block is empty); then the ratio candidate.  The objective row
// (local index rows) is current in place: C[j][rows] = z_q.
//
// Latency, not bytes, sets this kernel's time, so everything that does not
// depend on q is requested before the pricing reduce: the lane's whole replay
// chain of coefficients (from Cc, the column-major copy of C, so each load is
// one coalesced 512-B wave access), the RHS inputs, the basis entry, the step
// tables.  Only T0[i][q] and P[l][q] wait for q.  The workgroup partials are
// handed to the last-arriving workgroup without fences: write-through (sc1)
// stores drained by vmcnt(0) before the ticket add, sc1 loads after it
// (MI355X_MICROARCH.md, inter-workgroup visibility, first table row).
constexpr int kAuxSc1 = 16;   // buffer-op cache policy: sc1 (write-through store / L2 load)

// Fused single-rank pivot (pivot_defer_kernel): the workgroup that ends the ratio
// phase (the last arriver, or block 0 when nothing prices in) publishes the
// selection to the pivot-row workgroups of the same launch: st->zq, then an
// agent release and the flag st->go.
__device__ inline void release_go(DevState* st) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(&st->go, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Diagnostics (DLP_CHAIN_STAMPS=<file>, never set in a timed run): wall-clock stamps (100 MHz)
// of the phases of the lookahead chain kernels, one row per pivot (mod 64): ratio kernel
// workgroup 0 at start / q known / T0 and P[l][q] in / replay done / block reduce done /
// ticket taken, the last workgroup at its end; the pivot-row kernel's workgroup 0 at start /
// step table in / replay done / end.  Written by one lane; dumped by the session at free.
__device__ uint64_t g_chain_stamps[64][16];
__device__ int g_chain_stamps_on;
#define CHAIN_STAMP(slot, k)                                                                  \
    do {                                                                                      \
        if (g_chain_stamps_on && threadIdx.x == 0) g_chain_stamps[(slot) & 63][k] = wall_clock64(); \
    } while (0)
// Per-workgroup stamps of one selection per block (slot 40 mod 64; the grouped-ring kernel only):
// start / q known / T0 in / replay done / block reduce done / ticket taken, the CU (HW_ID), and
// wave 0's replayed steps (J - L0).
__device__ uint64_t g_wg_stamps[1024][8];
#define WG_STAMP(slot, k, v)                                                                   \
    do {                                                                                       \
        if (g_chain_stamps_on && threadIdx.x == 0 && ((slot) & 63) == 40 && blockIdx.x < 1024) \
            g_wg_stamps[blockIdx.x][k] = (v);                                                  \
    } while (0)

// LEAN (lookahead beside the form-21 pass): no register-resident chain (coefficients in
// pairs during the replay) and DPP wave minima for the block reductions (round 3: LDS trees),
// 30 VGPRs, so the kernel fits in the 32 VGPRs per SIMD that three pass waves (3 x 160) leave
// free.  Same operations in
// the same order.  (Staging the chain in LDS by LDS-DMA, 32 steps per round trip, measured
// no faster beside the pass: 96 vs 95 us per selection, profiles/r02j/.)
// LEAN, LCH = 0: the coefficient chain streams through a per-wave LDS ring by LDS-DMA, two
// steps per DMA, kRatioRingPairs DMAs in flight (launch-time LDS, kRatioRing bytes: see
// kProwRing).
// (RP = kRatioRingPairs: 16 measured equal at C3, 8,239-8,267 vs 8,262-8,263 pivots/s, profiles/r04c/)
constexpr int kRatioRingPairs = 8;
constexpr size_t ratio_ring_bytes(int rp) { return (size_t)(kRatioDeferThreads / 64) * rp * 128 * sizeof(double); }
// ROWS / RG (the ring only, round 6): ROWS rows per wave (64, 32, 16; 128 / ROWS steps per 1-KB
// DMA, lane x bringing step x / (ROWS / 2) of rows 2 (x % (ROWS / 2)), +1) and RG DMAs retired per
// wait, their LDS reads issued together: one wait and one LDS round trip per 2 RG (ROWS 64) steps
// instead of per pair.  A workgroup of blockDim.x lanes covers blockDim.x ROWS / 64 rows; lanes
// wl >= ROWS hold no row.  ROWS = 64, RG = 1 is the LEAN loop beside the pass.
template <int KMAX, bool FUSED, bool LEAN = false, int LCH = 4, int RP = kRatioRingPairs, bool DB = false,
          int ROWS = 64, int RG = 1>
__device__ __forceinline__ void ratio_defer_body(
    const double* __restrict__ T, int64_t ld, int64_t rows, int64_t rows_elig, int64_t ncols,
    int64_t row_first, int32_t* basis, const PricePart* __restrict__ pp, int ntiles,
    DevState* st, double* __restrict__ C, int64_t ldc, double* __restrict__ Cc, int64_t ldcc,
    const double* __restrict__ P, double* __restrict__ rhs, int32_t* __restrict__ nzc,
    Cand* partials, Cand* cand_out, int nranks, double tol_dj, double tol_piv, int pricing,
    dlp_pivot* log, int64_t log_cap, int nblocks, const double* __restrict__ Ccp = nullptr,
    const double* __restrict__ Pp = nullptr, int prev_seal = -1, const XPeers* xp = nullptr,
    uint32_t xseq = 0, uint32_t* bcnt = nullptr, int brb = 1, int bnt = 0, const double* Tn = nullptr,
    int xsel = 0, uint32_t rseq = 0, Cond cd = Cond{}) {
    // (the grouped ring reads up to 128 / ROWS * (RG + 1) table entries past J - 1, dropped)
    constexpr bool GRING = ROWS != 64 || RG != 1;
    constexpr int kPad = GRING ? 128 / ROWS * (RG + 1) : 0;
    constexpr int kWaves = GRING ? 16 : kRatioDeferThreads / 64;
    __shared__ PricePart lds_pp[kWaves];
    __shared__ Cand lds_c[kWaves];
    __shared__ int s_last;
    __shared__ double s_pq[KMAX + kPad], s_pn[KMAX];
    __shared__ int32_t s_pl[KMAX + kPad];
    auto cand_red = [&](Cand v) { return block_cand(v, lds_c); };
    // this lane's pricing partial is requested first: it depends on nothing, and the reduce
    // below then waits for it alongside the step-table loads instead of after them
    const PricePart pp0 = (int)threadIdx.x < ntiles ? pp[threadIdx.x] : pp_empty();
    if (st->status != DLP_RUNNING) return;
    const int64_t slot = st->npivots;
    if constexpr (LEAN) if (blockIdx.x == 0) CHAIN_STAMP(slot, 0);
    if constexpr (ROWS != 64 || RG != 1) WG_STAMP(slot, 0, wall_clock64());

    // replayed steps: the sealed previous block (lookahead: not yet applied to T, its kp
    // steps first), then this block's j steps; C / Cc / nzc are written at index j
    const int j = st->blk;
    const int kp = prev_seal >= 0 ? st->seal[prev_seal].blk : 0;
    const int J = kp + j;
    const int wl = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // the wave's rows [i0, i0 + ROWS); this lane's row i (none: far past every bound)
    const bool lane_row = !GRING || wl < ROWS;
    const int64_t i0 = GRING ? (int64_t)blockIdx.x * (blockDim.x / 64 * ROWS) + wv * ROWS
                             : (int64_t)blockIdx.x * blockDim.x + wv * 64;
    const int64_t i = !GRING ? (int64_t)blockIdx.x * blockDim.x + threadIdx.x
                             : (lane_row ? i0 + wl : ((int64_t)1 << 62));
    for (int l = threadIdx.x; l < J; l += blockDim.x) {
        s_pn[l] = l < kp ? Pp[(int64_t)l * ld + ncols] : P[(int64_t)(l - kp) * ld + ncols];
        s_pl[l] = l < kp ? st->seal[prev_seal].pl[l] : st->pl[l - kp];
    }
    // ring: lanes 0-31 of a DMA bring step 2p, lanes 32-63 step 2p+1, 16 B = two rows each,
    // so the ring slot holds the wave's 64 rows of both steps; Cc does not depend on q, so the
    // first DMAs are issued here and land during the pricing reduce.  Steps past J-1 re-read
    // step J-1 (harmless), so every pair issues exactly one DMA.
    constexpr bool RING = LEAN && LCH == 0;
    constexpr int SPD = 128 / ROWS, HL = ROWS / 2;   // steps per DMA; lanes per step
    extern __shared__ double s_dyn[];
    const bool wave_rows = i0 < rows;   // (i0 + ROWS - 1 < ldcc = round64(rows + 1))
    // band publication (RING): the wave's 64 rows final in Tn (their bands of the sealed
    // block's pass are done): start there and replay this block's steps only
    bool wdone = false;
    if constexpr (LEAN)
        if (bcnt && kp > 0 && i0 + ROWS - 1 < rows) {
            const int64_t b0 = i0 / brb, b1 = (i0 + ROWS - 1) / brb;
            const uint32_t c0 = __hip_atomic_load(&bcnt[b0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t c1 = b1 == b0 ? c0 : __hip_atomic_load(&bcnt[b1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            wdone = __builtin_amdgcn_readfirstlane(c0 == (uint32_t)bnt && c1 == (uint32_t)bnt ? 1 : 0) != 0;
        }
    const int L0 = wdone ? kp : 0;
    auto ring_at = [&](int p) { return s_dyn + (wv * RP + p % RP) * 128; };
    auto sbase = [&](int l) -> const double* {   // wave-uniform: step l's row i0 (l clamped)
        l = l < J ? l : J - 1;
        return (l < kp ? Ccp + (int64_t)l * ldcc : Cc + (int64_t)(l - kp) * ldcc) + i0;
    };
    auto csrc = [&](int p) -> const double* {
        if constexpr (ROWS == 64)
            return ((wl >> 5) ? sbase(L0 + 2 * p + 1) : sbase(L0 + 2 * p)) + 2 * (wl & 31);
        else
            return sbase(L0 + SPD * p + wl / HL) + 2 * (wl % HL);
    };
    if constexpr (RING)
        if (wave_rows && J > L0)
#pragma unroll
            for (int p = 0; p < RP; ++p) glds16(csrc(p), lds_addr(ring_at(p)));
    const int64_t ic = i < rows ? i : rows;   // clamped: loads need no guard
    double f[LEAN ? 1 : KMAX];
    if constexpr (!LEAN) {
#pragma unroll
        for (int l = 0; l < KMAX; ++l)
            f[l] = (l < J) ? (l < kp ? Ccp[(int64_t)l * ldcc + ic] : Cc[(int64_t)(l - kp) * ldcc + ic]) : 0.0;
    }
    auto fld = [&](int l) { return l < kp ? Ccp[(int64_t)l * ldcc + ic] : Cc[(int64_t)(l - kp) * ldcc + ic]; };
    double r_in = 0.0;
    int32_t nz_in = 0, bvar = 0;
    if (i < rows && j > 0) nz_in = nzc[i];
    if (i < rows_elig) {
        r_in = J == 0 ? T[i * ld + ncols] : rhs[i];
        bvar = basis[row_first + i];
    }

    PricePart acc = pp_empty();
    pp_combine(acc, pp0);
    for (int k = threadIdx.x + blockDim.x; k < ntiles; k += blockDim.x) pp_combine(acc, pp[k]);
    acc = block_price(acc, lds_pp);   // (DPP wave minima: LEAN too, within its 32 VGPRs)
    int32_t q;
    if (st->bland)
        q = acc.jbland;
    else
        q = (acc.jmin != kNoIndex && acc.zmin < -tol_dj) ? acc.jmin : kNoIndex;
    if (q == kNoIndex) {
        if constexpr (RING) vmwait<0>();   // no DMA into LDS outlives the wave
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            st->q = -1;
            st->status = DLP_OK;
            if constexpr (FUSED) release_go(st);
            if (xsel == 2) sel_publish(st, rseq, DLP_OK, 0.0);   // the pivot-row workgroups end too
        }
        return;
    }

    if constexpr (LEAN) if (blockIdx.x == 0) CHAIN_STAMP(slot, 1);
    if constexpr (GRING) WG_STAMP(slot, 1, wall_clock64());
    // condensed tableau: q's slot, and the step (of the replayed sequence: sealed steps first) at
    // which that slot restarted from the unit vector of its new variable (R < 0: none replayed here)
    // (the LCH = 8 tuning instance has no condensed build: its 32 VGPRs are full; the launcher
    // never picks it for a condensed session)
    int32_t sq = q, R = -1;
    if (!(LEAN && LCH == 8) && cd.on) {
        sq = __builtin_amdgcn_readfirstlane(cd.slot_of[q]);
        if (sq < 0 || sq >= ncols) {   // (an invariant: a priced variable is nonbasic) — never fault
            if constexpr (RING) vmwait<0>();
            if (blockIdx.x == 0 && threadIdx.x == 0) st->status = DLP_ERR_STATE;
            return;
        }
        const int32_t rv = __builtin_amdgcn_readfirstlane(cd.rst[sq]);
        if (rv >= 0) {
            if ((rv >> 7) == st->bser)
                R = kp + (rv & 127);
            else if (kp > 0 && (rv >> 7) == st->seal[prev_seal].ser)
                R = rv & 127;
        }
    }
    // T0[i][q] is requested before the P[l][q] loads and their barrier: both wait only for q
    double a = 0.0;
    if (wdone)   // sc1 load (the pass stored Tn write-through)
        a = __builtin_bit_cast(double, __hip_atomic_load((const uint64_t*)(Tn + i * ld + sq), __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT));
    else if (i <= rows)
        a = T[i * ld + sq];
    for (int l = threadIdx.x; l < J; l += blockDim.x)
        s_pq[l] = l < kp ? Pp[(int64_t)l * ld + sq] : P[(int64_t)(l - kp) * ld + sq];
    __syncthreads();
    if constexpr (LEAN) if (blockIdx.x == 0) CHAIN_STAMP(slot, 2);
    if constexpr (GRING) WG_STAMP(slot, 2, wall_clock64());

    Cand c = cand_empty();
    double flast = 0.0;   // LEAN: C of step J-1 (the RHS cache's step)
    if constexpr (RING) {
        // branch-free (the fma is computed and dropped where the eager rule skips it), so
        // the LDS reads of a pair's two steps issue together instead of one per branch
        // (ok = false: a pair's second step past J-1, read from the tables' spare entries and
        // dropped: l <= J <= KMAX - 1)
        // (condensed: at step R the slot's new column starts from the unit vector, +0 here)
        auto step = [&](int l, double fv, bool ok) {
            if (l == R) a = 0.0;   // (uniform; the objective row's lane reloads z_q below)
            const double pq = s_pq[l];
            const bool piv = i == s_pl[l];
            const double u = __builtin_fma(-fv, pq, a);
            a = ok && i < rows ? (piv ? pq : (fv != 0.0 ? u : a)) : a;
            flast = ok ? fv : flast;
        };
        if (wave_rows) {
            const int npairs = (J - L0 + SPD - 1) / SPD;   // (DMAs holding replayed steps)
            if constexpr (!GRING) {
                for (int p = 0; p < npairs; ++p) {
                    vmwait<RP - 1>();   // pair p landed: only ring DMAs issue in this loop
                    double* rs = ring_at(p);
                    const double f0 = rs[wl], f1 = rs[64 + wl];
                    step(L0 + 2 * p, f0, true);
                    step(L0 + 2 * p + 1, f1, L0 + 2 * p + 1 < J);
                    glds16(csrc(p + RP), lds_addr(rs));
                }
            } else {
                // RG DMAs per wait: their LDS reads together, then the SPD RG steps, then RG refills
                // (a group past the last DMA re-reads clamped steps, dropped: every group issues RG)
                const int r = wl % ROWS;
                for (int p0 = 0; p0 < npairs; p0 += RG) {
                    vmwait<RP - RG>();
                    double fq[SPD * RG];
#pragma unroll
                    for (int g = 0; g < RG; ++g) {
                        const double* rs = ring_at(p0 + g);
#pragma unroll
                        for (int k = 0; k < SPD; ++k) fq[g * SPD + k] = rs[k * ROWS + r];
                    }
#pragma unroll
                    for (int u = 0; u < SPD * RG; ++u) step(L0 + SPD * p0 + u, fq[u], L0 + SPD * p0 + u < J);
#pragma unroll
                    for (int g = 0; g < RG; ++g) glds16(csrc(p0 + g + RP), lds_addr(ring_at(p0 + g)));
                }
            }
            vmwait<0>();
            // no step replayed (first selection of a block on a finished band): the RHS cache
            // still advances by the sealed block's last step
            if (npairs == 0 && J > 0 && lane_row) flast = Ccp[(int64_t)(kp - 1) * ldcc + i];
            // (condensed: the restart step zeroed every lane of the wave; the objective row is
            // never replayed, its z_q is current)
            if (R >= L0 && i == rows) a = T[i * ld + sq];
        }
        if (blockIdx.x == 0) CHAIN_STAMP(slot, 3);
        if constexpr (GRING) {
            WG_STAMP(slot, 3, wall_clock64());
            WG_STAMP(slot, 6, (uint64_t)__smid());
            WG_STAMP(slot, 7, (uint64_t)(J - L0));
        }
    } else if constexpr (LEAN) {
        // LCH coefficient loads per round trip (the register budget of this kernel), from the
        // first step not applied to the row's source (L0: a published band starts after the
        // sealed block); the next chunk's loads are issued before this chunk is applied
        // (condensed: a restart of q's slot at R >= L0 starts the replay there from +0)
        const int Ls = R >= L0 ? R : L0;
        if (R >= L0 && i < rows) a = 0.0;
        if (i < rows && J > L0 && !DB) {   // one chunk at a time (LEAN's 32 VGPRs)
            for (int l0 = Ls; l0 < J; l0 += LCH) {
                double fq[LCH];
#pragma unroll
                for (int u = 0; u < LCH; ++u) fq[u] = l0 + u < J ? fld(l0 + u) : 0.0;
#pragma unroll
                for (int u = 0; u < LCH; ++u) {
                    const int l = l0 + u;
                    const double fv = fq[u];
                    if (l < J) {
                        if (i == s_pl[l])
                            a = s_pq[l];
                        else if (fv != 0.0)
                            a = __builtin_fma(-fv, s_pq[l], a);
                        flast = fv;
                    }
                }
            }
        } else if (i < rows && J > L0) {   // DB (MID): double-buffered
            double fa[LCH], fb[LCH];
            auto fetch = [&](double (&fq)[LCH], int l0) {
#pragma unroll
                for (int u = 0; u < LCH; ++u) fq[u] = l0 + u < J ? fld(l0 + u) : 0.0;
            };
            auto apply = [&](const double (&fq)[LCH], int l0) {
#pragma unroll
                for (int u = 0; u < LCH; ++u) {
                    const int l = l0 + u;
                    const double fv = fq[u];
                    if (l < J) {
                        if (i == s_pl[l])
                            a = s_pq[l];
                        else if (fv != 0.0)
                            a = __builtin_fma(-fv, s_pq[l], a);
                        flast = fv;
                    }
                }
            };
            fetch(fa, Ls);
            for (int l0 = Ls; l0 < J; l0 += 2 * LCH) {
                if (l0 + LCH < J) fetch(fb, l0 + LCH);
                apply(fa, l0);
                if (l0 + LCH >= J) break;
                if (l0 + 2 * LCH < J) fetch(fa, l0 + 2 * LCH);
                apply(fb, l0 + LCH);
            }
        } else if (i < rows && J > 0 && L0 == J) {
            flast = Ccp[(int64_t)(kp - 1) * ldcc + i];   // nothing replayed: the RHS cache's step
        }
        if (blockIdx.x == 0) CHAIN_STAMP(slot, 3);
    }
    if (i <= rows) {
        if (i < rows) {
            if constexpr (!LEAN) {   // (LEAN replayed above)
#pragma unroll
                for (int l = 0; l < KMAX; ++l) {
                    if (l < J) {
                        if (l == R) a = 0.0;
                        if (i == s_pl[l])
                            a = s_pq[l];
                        else if (f[l] != 0.0)
                            a = __builtin_fma(-f[l], s_pq[l], a);
                    }
                }
            }
        }
        C[i * ldc + j] = a;
        // block start: the row's coefficients of steps 1..K-1 := +0, so a pass over a partial
        // block (kb < K steps) runs the full-block code: P[l >= kb] is +0 too (commit_row),
        // and fma(-(+0), +0, t) = t + (-0) = t for every t
        if (j == 0)
            for (int64_t l = 1; l < ldc; ++l) C[i * ldc + l] = 0.0;
        Cc[(int64_t)j * ldcc + i] = a;
        if (i < rows) nzc[i] = (j == 0 ? 0 : nz_in) + (a != 0.0 ? 1 : 0);   // the pass's row class
        if (i < rows_elig) {
            double r = r_in;
            if (J > 0) {
                const int l = J - 1;
                double fp = 0.0;   // f[j-1], selected without dynamic register indexing
                if constexpr (LEAN) {
                    fp = flast;
                } else {
#pragma unroll
                    for (int u = 0; u < KMAX; ++u) fp = (u == l) ? f[u] : fp;
                }
                if (i == s_pl[l])
                    r = s_pn[l];
                else if (fp != 0.0)
                    r = __builtin_fma(-fp, s_pn[l], r);
            }
            rhs[i] = r;
            if (a > tol_piv) {
                double b = r;
                if (!(b > 0.0)) b = 0.0;
                c.ratio = b / a;
                c.row = (int32_t)(row_first + i);
                c.basis_var = bvar;
                c.valid = 1;
                c.pivot = a;
            }
        }
    }
    c = cand_red(c);
    if constexpr (LEAN) if (blockIdx.x == 0) CHAIN_STAMP(slot, 4);
    if constexpr (GRING) WG_STAMP(slot, 4, wall_clock64());
    if (xp && xsel) {
        // peer exchange, selection in this launch: every workgroup's candidate straight into slot
        // [seq & 1][me][blockIdx] of every rank (no partials, no ticket); workgroup 0 of every rank
        // waits for all of them, reduces them in the candidate order and selects (every rank
        // reaches the same p).  A workgroup's reads of the state are done before it pushes, so the
        // selection never races them.
        if (threadIdx.x == 0) x_push_cand(xp, xseq, c, (int)blockIdx.x);
        if (blockIdx.x != 0) return;
        __shared__ int s_xok;
        Cand w;
        if (!x_gather_all(xp, xseq, &w, &s_xok)) {
            if (threadIdx.x == 0) {
                st->status = kStatusXFail;
                if (xsel == 2) sel_publish(st, rseq, kStatusXFail, 0.0);
            }
            return;
        }
        w = cand_red(w);
        if (threadIdx.x == 0) {
            // one-launch pivot: z_q (the objective row is current; this launch's commit writes it
            // only after the record) before the selection, which writes the log entry's other fields
            const double zq = xsel == 2 ? T[rows * ld + sq] : 0.0;
            st->sq = sq;
            do_select(st, w, q, basis, row_first, rows, pricing, log, log_cap, true, xsel != 2, cd);
            if (xsel == 2) sel_publish(st, rseq, st->status, zq);
        }
        if constexpr (LEAN) CHAIN_STAMP(slot, 6);
        return;
    }

    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)partials, (short)0, (int)(nblocks * sizeof(Cand)), 0x00020000);
    if (threadIdx.x == 0) {
        const u4v* cv = (const u4v*)&c;
        __builtin_amdgcn_raw_buffer_store_b128(cv[0], prs, (int)(blockIdx.x * sizeof(Cand)), 0, kAuxSc1);
        __builtin_amdgcn_raw_buffer_store_b128(cv[1], prs, (int)(blockIdx.x * sizeof(Cand)) + 16, 0,
                                               kAuxSc1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned prev =
            __hip_atomic_fetch_add(&st->ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = (prev == (unsigned)nblocks - 1);
    }
    __syncthreads();
    if constexpr (LEAN) if (blockIdx.x == 0) CHAIN_STAMP(slot, 5);
    if constexpr (GRING) WG_STAMP(slot, 5, wall_clock64());
    if (!s_last) return;
    Cand best = cand_empty();
    for (int k = threadIdx.x; k < nblocks; k += blockDim.x) {
        Cand o;
        u4v* ov = (u4v*)&o;
        ov[0] = __builtin_amdgcn_raw_buffer_load_b128(prs, (int)(k * sizeof(Cand)), 0, kAuxSc1);
        ov[1] = __builtin_amdgcn_raw_buffer_load_b128(prs, (int)(k * sizeof(Cand)) + 16, 0, kAuxSc1);
        if (cand_better(o, best)) best = o;
    }
    best = cand_red(best);
    if (threadIdx.x == 0) {
        st->ticket = 0;
        st->q = q;
        st->sq = sq;
        if (nranks == 1)
            do_select(st, best, q, basis, row_first, rows, pricing, log, log_cap, true, true, cd);
        else if (xp)
            x_push_cand(xp, xseq, best);   // peer exchange: straight into every rank's slot
        else
            cand_out[0] = best;
        if constexpr (FUSED) {
            st->zq = T[rows * ld + sq];   // the objective row is current; nobody writes it yet
            release_go(st);
        }
    }

    if constexpr (LEAN) CHAIN_STAMP(slot, 6);
}

template <int KMAX>
__global__ __launch_bounds__(kRatioDeferThreads) void ratio_defer_kernel(
    const double* __restrict__ T, int64_t ld, int64_t rows, int64_t rows_elig, int64_t ncols,
    int64_t row_first, int32_t* basis, const PricePart* __restrict__ pp, int ntiles,
    DevState* st, double* __restrict__ C, int64_t ldc, double* __restrict__ Cc, int64_t ldcc,
    const double* __restrict__ P, double* __restrict__ rhs, int32_t* __restrict__ nzc,
    Cand* partials, Cand* cand_out, int nranks, double tol_dj, double tol_piv, int pricing,
    dlp_pivot* log, int64_t log_cap, const double* __restrict__ Ccp, const double* __restrict__ Pp,
    int prev_seal, const XPeers* xp, uint32_t xseq, int xsel, Cond cd) {
    ratio_defer_body<KMAX, false>(T, ld, rows, rows_elig, ncols, row_first, basis, pp, ntiles, st, C,
                                  ldc, Cc, ldcc, P, rhs, nzc, partials, cand_out, nranks, tol_dj,
                                  tol_piv, pricing, log, log_cap, (int)gridDim.x, Ccp, Pp, prev_seal,
                                  xp, xseq, nullptr, 1, 0, nullptr, xsel, 0, cd);
}

// MID (round 5): beside the MFMA pass (form 22 leaves 104 VGPRs per SIMD), the replay's
// coefficients in registers, LCH per round trip, double-buffered, no LDS ring.
template <int KMAX, int LCH>
__global__ __launch_bounds__(kRatioDeferThreads) __attribute__((amdgpu_num_vgpr(104))) void ratio_mid_kernel(
    const double* __restrict__ T, int64_t ld, int64_t rows, int64_t rows_elig, int64_t ncols,
    int64_t row_first, int32_t* basis, const PricePart* __restrict__ pp, int ntiles,
    DevState* st, double* __restrict__ C, int64_t ldc, double* __restrict__ Cc, int64_t ldcc,
    const double* __restrict__ P, double* __restrict__ rhs, int32_t* __restrict__ nzc,
    Cand* partials, Cand* cand_out, int nranks, double tol_dj, double tol_piv, int pricing,
    dlp_pivot* log, int64_t log_cap, const double* __restrict__ Ccp, const double* __restrict__ Pp,
    int prev_seal, const XPeers* xp, uint32_t xseq, uint32_t* bcnt, int brb, int bnt, const double* Tn,
    int xsel, Cond cd) {
    ratio_defer_body<KMAX, false, true, LCH, kRatioRingPairs, true>(T, ld, rows, rows_elig, ncols, row_first, basis, pp, ntiles, st, C,
                                             ldc, Cc, ldcc, P, rhs, nzc, partials, cand_out, nranks, tol_dj,
                                             tol_piv, pricing, log, log_cap, (int)gridDim.x, Ccp, Pp, prev_seal,
                                             xp, xseq, bcnt, brb, bnt, Tn, xsel, 0, cd);
}

// The LEAN selection kernel, held to 32 VGPRs (lookahead at K = 64, beside the pass).
template <int KMAX, int LCH, int RP = kRatioRingPairs>
__global__ __launch_bounds__(kRatioDeferThreads) __attribute__((amdgpu_num_vgpr(32))) void ratio_lean_kernel(
    const double* __restrict__ T, int64_t ld, int64_t rows, int64_t rows_elig, int64_t ncols,
    int64_t row_first, int32_t* basis, const PricePart* __restrict__ pp, int ntiles,
    DevState* st, double* __restrict__ C, int64_t ldc, double* __restrict__ Cc, int64_t ldcc,
    const double* __restrict__ P, double* __restrict__ rhs, int32_t* __restrict__ nzc,
    Cand* partials, Cand* cand_out, int nranks, double tol_dj, double tol_piv, int pricing,
    dlp_pivot* log, int64_t log_cap, const double* __restrict__ Ccp, const double* __restrict__ Pp,
    int prev_seal, const XPeers* xp, uint32_t xseq, uint32_t* bcnt, int brb, int bnt, const double* Tn,
    int xsel, Cond cd) {
    ratio_defer_body<KMAX, false, true, LCH, RP>(T, ld, rows, rows_elig, ncols, row_first, basis, pp, ntiles, st, C,
                                        ldc, Cc, ldcc, P, rhs, nzc, partials, cand_out, nranks, tol_dj,
                                        tol_piv, pricing, log, log_cap, (int)gridDim.x, Ccp, Pp, prev_seal,
                                        xp, xseq, bcnt, brb, bnt, Tn, xsel, 0, cd);
}

// The grouped ring (round 6): the selection kernel of a chain on CUs of its own (the lookahead's
// disjoint CU masks: no pass waves beside it, so no 32-VGPR budget).  ROWS rows per wave, RP DMAs
// in flight, RG retired per wait (tools/chainlab.hip, profiles/r06q/-r06s/).  Launched with
// rthreads x 64 / ROWS lanes, so a workgroup covers the session's rthreads rows and the grid, the
// partials and the exchange's candidate slots are those of every other ratio kernel.
template <int ROWS, int RP, int RG>
__global__ __launch_bounds__(1024) void ratio_ring_kernel(
    const double* __restrict__ T, int64_t ld, int64_t rows, int64_t rows_elig, int64_t ncols,
    int64_t row_first, int32_t* basis, const PricePart* __restrict__ pp, int ntiles,
    DevState* st, double* __restrict__ C, int64_t ldc, double* __restrict__ Cc, int64_t ldcc,
    const double* __restrict__ P, double* __restrict__ rhs, int32_t* __restrict__ nzc,
    Cand* partials, Cand* cand_out, int nranks, double tol_dj, double tol_piv, int pricing,
    dlp_pivot* log, int64_t log_cap, const double* __restrict__ Ccp, const double* __restrict__ Pp,
    int prev_seal, const XPeers* xp, uint32_t xseq, uint32_t* bcnt, int brb, int bnt, const double* Tn,
    int xsel, Cond cd) {
    ratio_defer_body<128, false, true, 0, RP, false, ROWS, RG>(
        T, ld, rows, rows_elig, ncols, row_first, basis, pp, ntiles, st, C, ldc, Cc, ldcc, P, rhs, nzc, partials,
        cand_out, nranks, tol_dj, tol_piv, pricing, log, log_cap, (int)gridDim.x, Ccp, Pp, prev_seal, xp, xseq, bcnt,
        brb, bnt, Tn, xsel, 0, cd);
}

// P[s] := pr for columns j, j+1; objective row z -= z_q * P[s] (z_q != 0);
// pricing partial of this 512-column tile (pp[tile]); objective value into log[klog].
// Same per-element operations as the eager update kernel's objective band.
// ZQ: 0 = z_q from C[rows][s]; 1 = the caller's early loads of T[rows][j..j+1] (zpre) and z_q
// (zqv); 2 = z_q given (zqv: the selection record of a one-launch pivot), z loaded here
// Condensed tableau (cd.on): slot sq is the entering variable's, now the leaving variable's: its
// objective entry restarts from +0 (a basic column's), its restart is recorded (rst, block
// serial bser, step s) and its entries of the block's earlier pivot rows become +0 (the pass
// starts the slot from the unit vector written by reset_cols); pricing by variable (var_of).
template <int ZQ = 0>
__device__ inline void commit_row(double* __restrict__ T, int64_t ld, int64_t rows, int64_t ncols,
                                  int64_t nprice, int64_t klog, const double* __restrict__ C,
                                  int64_t ldc, double* __restrict__ P, int s, int64_t j, d2 pr,
                                  PricePart* pp, int tile, double tol_dj, dlp_pivot* log, int64_t log_cap,
                                  PricePart* lds_pp, d2 zpre = d2{0.0, 0.0}, double zqv = 0.0,
                                  Cond cd = Cond{}, int32_t sq = -1, int32_t bser = 0) {
    const int64_t width = (ncols + 16) & ~(int64_t)15;
    const bool rx = cd.on && j == sq, ry = cd.on && j + 1 == sq;
    if (j < ld) {
        *(d2*)(P + (int64_t)s * ld + j) = pr;
        if (s == 0)   // block start: pivot rows 1..K-1 := +0 (see the ratio kernel's C tails)
            for (int64_t l = 1; l < ldc; ++l) *(d2*)(P + l * ld + j) = d2{0.0, 0.0};
        if (rx || ry) {
            for (int l = 0; l < s; ++l) P[(int64_t)l * ld + sq] = 0.0;
            cd.rst[sq] = (bser << 7) | s;
        }
    }
    const double zq = ZQ == 0 ? C[rows * ldc + s] : zqv;
    PricePart acc = pp_empty();
    if (j < width) {
        double* zp = T + rows * ld + j;
        d2 z = ZQ == 1 ? zpre : *(const d2*)zp;
        if (rx) z.x = 0.0;
        if (ry) z.y = 0.0;
        if (zq != 0.0) {
            z.x = __builtin_fma(-zq, pr.x, z.x);
            z.y = __builtin_fma(-zq, pr.y, z.y);
        }
        if (zq != 0.0 || rx || ry) *(d2*)zp = z;
        if (cd.on)
            price_pair_var(acc, z.x, z.y, cd.var_of[j], cd.var_of[j + 1], tol_dj);
        else
            price_pair(acc, z.x, z.y, j, nprice, tol_dj);
        if (log && j <= ncols && ncols < j + 2) {
            if (klog >= 0 && klog < log_cap) log[klog].objective = (ncols == j) ? z.x : z.y;
        }
    }
    acc = block_price(acc, lds_pp);
    if (threadIdx.x == 0) pp[tile] = acc;
}

// a3 first half on the replayed pivot row: T_s[p] = steps 0..s-1 applied to
// T0[p], divided by the pivot element (IEEE division).  fused (single rank):
// commit_row as well.  Otherwise the owner writes the fp64 bits and every
// other rank INT64_MIN for the int64 MAX exchange.
constexpr int kProwRingSteps = 8;   // (RS: 16 measured equal, with the ratio ring's 16)
constexpr size_t prow_ring_bytes(int rs) { return (size_t)4 * rs * 128 * sizeof(double); }
// PG (the ring only, round 6): pivot rows retired per wait, their LDS reads issued together (PG = 1:
// one wait and one LDS round trip per row, the 32-VGPR kernel beside the pass)
template <bool LEAN, int RS = kProwRingSteps, int CHR = 16, int PG = 1>
__device__ __forceinline__ void prow_defer_body(
    double* __restrict__ T, int64_t ld, int64_t rows, int64_t ncols, int64_t nprice,
    const DevState* st, const double* __restrict__ C, int64_t ldc, double* __restrict__ P,
    int64_t* __restrict__ bits, PricePart* pp, double tol_dj, dlp_pivot* log, int64_t log_cap,
    int fused, const double* __restrict__ Cp, const double* __restrict__ Pp, int prev_seal,
    const XPeers* xp, uint32_t xseq, uint32_t* bcnt, int brb, int bnt, const double* Tn, int xcommit,
    int tile, int onelaunch = 0, Cond cd = Cond{}) {
    __shared__ PricePart lds_pp[4];
    __shared__ SelView s_sel;
    __shared__ int s_selok;
    __shared__ double s_cp[kMaxReplay + (PG > 1 ? PG : 0)];   // (a group past S - 1 reads spares, dropped)
    __shared__ int32_t s_pl[kMaxReplay + (PG > 1 ? PG : 0)];
    // LEAN: the replayed pivot rows stream through a per-wave LDS ring by LDS-DMA, RING steps
    // in flight (each lane's own 16 B of a row land at ring + 16 lane), instead of 4 rows per
    // round trip in the 32 VGPRs this kernel has beside the pass
    // (launch-time LDS, kProwRing bytes: static LDS of that size makes hipcc's descriptor ask for
    // the VGPRs its LDS-bound occupancy would leave, 176, and the kernel no longer fits beside
    // the pass)
    constexpr int RING = RS;
    extern __shared__ double s_dyn[];
    auto s_ring = reinterpret_cast<double(*)[RING][128]>(s_dyn);
    if (st->status != DLP_RUNNING) return;   // an earlier launch ended the solve
    // the selection: from the state (a launch of its own), or, in a one-launch pivot (peer
    // exchange), from the record the ratio workgroups of this launch publish (DevState::SelRec)
    SelView sv;
    if (onelaunch) {
        if (!sel_wait(xp, st, xseq, &sv, &s_sel, &s_selok)) {
            if (threadIdx.x == 0) const_cast<DevState*>(st)->status = kStatusXFail;   // (writable memory)
            return;
        }
        if (sv.status != DLP_RUNNING) return;
    } else {
        sv.status = DLP_RUNNING;
        sv.p_local = st->p_local;
        sv.blk = st->blk;
        sv.piv = st->piv;
        sv.zq = 0.0;
        sv.npivots = st->npivots;
        sv.sq = -1;
    }
    const int64_t slot = sv.npivots - 1;
    if constexpr (LEAN) if (tile == 0) CHAIN_STAMP(slot, 8);
    const int s = sv.blk - 1;
    // replayed steps: the sealed previous block first (lookahead), then this block's s
    const int kp = prev_seal >= 0 ? st->seal[prev_seal].blk : 0;
    const int S = kp + s;
    const int32_t pl = sv.p_local;
    const int64_t j = ((int64_t)tile * blockDim.x + threadIdx.x) * 2;
    const bool owner_lane = pl >= 0 && j < ld;
    // LEAN, band publication: row p final in Tn (its band of the sealed block's pass is done):
    // start there and replay this block's steps only
    bool pdone = false;
    if (bcnt && kp > 0 && pl >= 0)
            pdone = __builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(&bcnt[pl / brb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == (uint32_t)bnt;
    const int L0 = pdone ? kp : 0;
    // the ring's first RING rows are requested first (they depend on nothing but the step
    // counts); rows past the last step re-read it (harmless), so every step issues one DMA
    auto psrc = [&](int l) -> const double* {
        l = l < S ? l : S - 1;
        return (l < kp ? Pp + (int64_t)l * ld : P + (int64_t)(l - kp) * ld) + j;
    };
    const int wv = threadIdx.x >> 6, wl = threadIdx.x & 63;
    if constexpr (LEAN)
        if (owner_lane && S > L0)
#pragma unroll
            for (int r = 0; r < RING; ++r) glds16(psrc(L0 + r), lds_addr(&s_ring[wv][(L0 + r) % RING][0]));
    // everything that depends only on (p, s) is requested before the step-table barrier:
    // T0[p][j..j+1] and, for the fused commit, the objective row and z_q
    d2 t0 = d2{0.0, 0.0}, zpre = d2{0.0, 0.0};
    double zqpre = 0.0;
    if (pdone && j < ld) {   // sc1 loads (the pass stored Tn write-through)
        const uint64_t* tn = (const uint64_t*)(Tn + (int64_t)pl * ld + j);
        const double x0 = __builtin_bit_cast(double, __hip_atomic_load(tn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const double x1 = __builtin_bit_cast(double, __hip_atomic_load(tn + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        t0.x = x0;
        t0.y = x1;
    } else if (pl >= 0 && j < ld) {
        t0 = *(const d2*)(T + (int64_t)pl * ld + j);
    }
    // condensed tableau: the lane's two slots' restarts (the step of the replayed sequence at which
    // each restarts from +0, -1: none here) and the entering slot (its entry of row p is the
    // leaving variable's unit 1)
    int32_t Rx = -1, Ry = -1, sq = -1;
    if (cd.on) {
        sq = onelaunch ? sv.sq : st->sq;   // (one launch: the record's, published with the selection)
        if (owner_lane) {
            const int bs = st->bser, ss = kp > 0 ? st->seal[prev_seal].ser : -2;
            // (a sealed-block restart matters only where row p is replayed through the sealed
            // block: a published row p already holds its result)
            auto rof = [&](int32_t rv) -> int32_t {
                if (rv < 0) return -1;
                if ((rv >> 7) == bs) return kp + (rv & 127);
                return (!pdone && (rv >> 7) == ss) ? (rv & 127) : -1;
            };
            Rx = rof(cd.rst[j]);
            Ry = rof(cd.rst[j + 1]);
        }
    }
    // The restarts: inside the replay loops (the slot's value becomes +0 at its restart step), or,
    // in the MID instance (CHR 8), whose registers are budgeted beside the MFMA pass, after the
    // loop: a restarted slot is replayed again from +0 at its restart step, its pivot rows from
    // global memory.  Then the entering slot's entry is the leaving variable's unit 1.
    constexpr bool kFixAfter = !LEAN && CHR == 8;
    auto cond_fix = [&](d2& t) {
        if (kFixAfter && (Rx >= 0 || Ry >= 0)) {
            const int r0 = Rx < 0 ? Ry : (Ry < 0 ? Rx : min(Rx, Ry));
            if (Rx >= 0) t.x = 0.0;
            if (Ry >= 0) t.y = 0.0;
            for (int l = r0; l < S; ++l) {
                const d2 pv = *(const d2*)((l < kp ? Pp + (int64_t)l * ld : P + (int64_t)(l - kp) * ld) + j);
                const double cp = s_cp[l];
                const bool piv = pl == s_pl[l];
                if (Rx >= 0 && l >= Rx) t.x = piv ? pv.x : (cp != 0.0 ? __builtin_fma(-cp, pv.x, t.x) : t.x);
                if (Ry >= 0 && l >= Ry) t.y = piv ? pv.y : (cp != 0.0 ? __builtin_fma(-cp, pv.y, t.y) : t.y);
            }
        }
        if (j == sq) t.x = 1.0;
        if (j + 1 == sq) t.y = 1.0;
    };
    if (fused && !LEAN) {   // (LEAN: within the 32 VGPRs that let it run beside the pass)
        zqpre = C[rows * ldc + s];
        if (j < ((ncols + 16) & ~(int64_t)15)) zpre = *(const d2*)(T + rows * ld + j);
    }
    if (pl >= 0)
        for (int l = threadIdx.x; l < S; l += blockDim.x) {
            s_cp[l] = l < kp ? Cp[(int64_t)pl * ldc + l] : C[(int64_t)pl * ldc + (l - kp)];
            s_pl[l] = l < kp ? st->seal[prev_seal].pl[l] : st->pl[l - kp];
        }
    __syncthreads();
    if constexpr (LEAN) if (tile == 0) CHAIN_STAMP(slot, 9);
    d2 pr;
    pr.x = 0.0;
    pr.y = 0.0;
    if (owner_lane && LEAN) {
        d2 t = t0;
        asm volatile("" ::"v"(t.x), "v"(t.y));   // T0[p] in here (hipcc's own wait), not in the loop
        if constexpr (PG == 1) {
            for (int l = L0; l < S; ++l) {
                vmwait<RING - 1>();   // step l's DMA retired: only ring DMAs issue in this loop
                const d2 pv = *(const d2*)&s_ring[wv][l % RING][2 * wl];
                const double cp = s_cp[l];
                const bool piv = pl == s_pl[l];
                if (l == Rx) t.x = 0.0;
                if (l == Ry) t.y = 0.0;
                const double ux = __builtin_fma(-cp, pv.x, t.x), uy = __builtin_fma(-cp, pv.y, t.y);
                t.x = piv ? pv.x : (cp != 0.0 ? ux : t.x);   // (branch-free, as the ratio ring's step)
                t.y = piv ? pv.y : (cp != 0.0 ? uy : t.y);
                glds16(psrc(l + RING), lds_addr(&s_ring[wv][l % RING][0]));
            }
        } else {
            // PG rows per wait: their LDS reads together, then the PG steps, then PG refills (a group
            // past S - 1 reads clamped rows and drops them: every group issues PG DMAs)
            for (int l0 = L0; l0 < S; l0 += PG) {
                vmwait<RING - PG>();
                d2 pv[PG];
#pragma unroll
                for (int g = 0; g < PG; ++g) pv[g] = *(const d2*)&s_ring[wv][(l0 + g) % RING][2 * wl];
#pragma unroll
                for (int g = 0; g < PG; ++g) {
                    const int l = l0 + g;
                    const double cp = s_cp[l];
                    const bool piv = pl == s_pl[l];
                    const bool ok = l < S;
                    if (l == Rx) t.x = 0.0;
                    if (l == Ry) t.y = 0.0;
                    const double ux = __builtin_fma(-cp, pv[g].x, t.x), uy = __builtin_fma(-cp, pv[g].y, t.y);
                    t.x = ok ? (piv ? pv[g].x : (cp != 0.0 ? ux : t.x)) : t.x;
                    t.y = ok ? (piv ? pv[g].y : (cp != 0.0 ? uy : t.y)) : t.y;
                }
#pragma unroll
                for (int g = 0; g < PG; ++g) glds16(psrc(l0 + g + RING), lds_addr(&s_ring[wv][(l0 + g) % RING][0]));
            }
        }
        vmwait<0>();   // the ring drained (the clamped tail DMAs) before the block exits
        if (cd.on) cond_fix(t);
        const double piv = sv.piv;
        pr.x = t.x / piv;
        pr.y = t.y / piv;
    } else if (owner_lane) {
        d2 t = t0;
        // chunks of CH pivot rows (row index clamped), double-buffered: the next chunk's loads are
        // issued before this chunk is applied, so up to 2 CH rows are in flight (c3r8: the replay
        // was 7 us per pivot with one chunk of 8 in flight, profiles/r04e/)
        constexpr int CH = CHR;
        d2 pa[CH], pb[CH];
        auto fetch = [&](d2 (&pv)[CH], int l0) {
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int l = min(l0 + u, S - 1);
                pv[u] = *(const d2*)((l < kp ? Pp + (int64_t)l * ld : P + (int64_t)(l - kp) * ld) + j);
            }
        };
        auto apply = [&](const d2 (&pv)[CH], int l0) {
#pragma unroll
            for (int u = 0; u < CH; ++u) {
                const int l = l0 + u;
                if (l < S) {
                    if (!kFixAfter && l == Rx) t.x = 0.0;
                    if (!kFixAfter && l == Ry) t.y = 0.0;
                    if (pl == s_pl[l]) {
                        t = pv[u];
                    } else if (s_cp[l] != 0.0) {
                        t.x = __builtin_fma(-s_cp[l], pv[u].x, t.x);
                        t.y = __builtin_fma(-s_cp[l], pv[u].y, t.y);
                    }
                }
            }
        };
        if (S > L0) fetch(pa, L0);
        for (int l0 = L0; l0 < S; l0 += 2 * CH) {
            if (l0 + CH < S) fetch(pb, l0 + CH);
            apply(pa, l0);
            if (l0 + CH >= S) break;
            if (l0 + 2 * CH < S) fetch(pa, l0 + 2 * CH);
            apply(pb, l0 + CH);
        }
        if (cd.on) cond_fix(t);
        const double piv = sv.piv;
        pr.x = t.x / piv;
        pr.y = t.y / piv;
    }
    if constexpr (LEAN) if (tile == 0) CHAIN_STAMP(slot, 10);
    if (!fused && xp) {   // peer exchange: the owner's row into every rank's row region
        // (scalars first: hipcc of ROCm 7.2 compiles __builtin_bit_cast(T, v.y) of an
        // ext_vector element as a cast of element 0; tests/test_isa.py guards this site)
        const double px = pr.x, py = pr.y;
        if (pl >= 0)      // (uniform per launch)
            x_push_row_chunk(xp, xseq, j, ld, __builtin_bit_cast(uint64_t, px),
                             __builtin_bit_cast(uint64_t, py), tile);
        if constexpr (LEAN) if (tile == 0) CHAIN_STAMP(slot, 11);
        if (!xcommit) return;
        // the commit in this launch (no commit launch): the owner commits the row it holds, every
        // other rank waits for this chunk's flag and reads the chunk from its own row region
        if (pl < 0) {
            __shared__ int s_xok;
            if (threadIdx.x == 0) s_xok = x_wait(xp, x_rflag(xp, xp->me, tile), xseq) ? 1 : 0;
            __syncthreads();
            if (!s_xok) {
                if (threadIdx.x == 0) const_cast<DevState*>(st)->status = kStatusXFail;   // (st is writable memory)
                return;
            }
            if (j < ld) {
                uint64_t a = 0, b = 0;
                x_read_row_pair(xp, j, &a, &b);
                pr.x = __builtin_bit_cast(double, a);
                pr.y = __builtin_bit_cast(double, b);
            }
        }
        if constexpr (LEAN) if (tile == 0) CHAIN_STAMP(slot, 13);
        if (onelaunch)   // z_q from the record (C[rows][s] is another workgroup's store of this launch)
            commit_row<2>(T, ld, rows, ncols, nprice, slot, C, ldc, P, s, j, pr, pp, tile, tol_dj, log, log_cap,
                          lds_pp, d2{0.0, 0.0}, sv.zq, cd, sq, cd.on ? st->bser : 0);
        else
            commit_row(T, ld, rows, ncols, nprice, slot, C, ldc, P, s, j, pr, pp, tile, tol_dj, log, log_cap, lds_pp,
                       d2{0.0, 0.0}, 0.0, cd, sq, cd.on ? st->bser : 0);
        if constexpr (LEAN) if (tile == 0) CHAIN_STAMP(slot, 14);
        return;
    }
    if (!fused) {
        if (j < ld) {
            if (pl >= 0) {
                *(d2*)(bits + j) = pr;   // the fp64 bits, as int64
            } else {
                bits[j] = INT64_MIN;
                bits[j + 1] = INT64_MIN;
            }
        }
        return;
    }
    commit_row<LEAN ? 0 : 1>(T, ld, rows, ncols, nprice, slot, C, ldc, P, s, j, pr, pp, tile, tol_dj, log,
                             log_cap, lds_pp, zpre, zqpre, cd, sq, cd.on ? st->bser : 0);
    if constexpr (LEAN) if (tile == 0) CHAIN_STAMP(slot, 11);
}
#define DLP_PROW_ARGS                                                                              \
    double *__restrict__ T, int64_t ld, int64_t rows, int64_t ncols, int64_t nprice, const DevState *st, \
        const double *__restrict__ C, int64_t ldc, double *__restrict__ P, int64_t *__restrict__ bits,  \
        PricePart *pp, double tol_dj, dlp_pivot *log, int64_t log_cap, int fused,                    \
        const double *__restrict__ Cp, const double *__restrict__ Pp, int prev_seal, const XPeers *xp, \
        uint32_t xseq, uint32_t *bcnt, int brb, int bnt, const double *Tn, int xcommit, Cond cd
#define DLP_PROW_PASS T, ld, rows, ncols, nprice, st, C, ldc, P, bits, pp, tol_dj, log, log_cap, fused, Cp, Pp, \
                      prev_seal, xp, xseq, bcnt, brb, bnt, Tn, xcommit, (int)blockIdx.x, 0, cd
// The LEAN instance (lookahead at K = 64, beside the form-21 pass) is held to 32 VGPRs in its
// kernel descriptor: the pass leaves 32 per SIMD (with the LDS-DMA asm, hipcc's descriptor
// otherwise requested 176 for a body that uses 30, and the kernel could not share a CU).
template <bool LEAN = false>
__global__ __launch_bounds__(256) void prow_defer_kernel(DLP_PROW_ARGS) {
    prow_defer_body<false>(DLP_PROW_PASS);
}
template <int RS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(32))) void prow_lean_kernel(DLP_PROW_ARGS) {
    prow_defer_body<true, RS>(DLP_PROW_PASS);
}
// The grouped ring (round 6): the pivot-row kernel of a chain on CUs of its own, RS rows in flight,
// PG retired per wait (no 32-VGPR budget: no pass waves beside it)
template <int RS, int PG>
__global__ __launch_bounds__(256) void prow_ring_kernel(DLP_PROW_ARGS) {
    prow_defer_body<true, RS, 16, PG>(DLP_PROW_PASS);
}
// MID (round 5): beside the MFMA pass (form 22: 3 waves x 136 VGPRs per SIMD leave 104), the
// register replay of the fat kernel with 2 x 8 pivot rows in flight instead of 2 x 16, and no
// LDS ring (the MFMA pass stages its coefficients through LDS).
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(104))) void prow_mid_kernel(DLP_PROW_ARGS) {
    prow_defer_body<false, kProwRingSteps, 8>(DLP_PROW_PASS);
}
#undef DLP_PROW_ARGS
#undef DLP_PROW_PASS

// Peer exchange, one launch per pivot (dlp::launch_pivot_x): workgroups [0, nrat) run the ratio
// test and the selection (every workgroup pushes its candidate to every rank, workgroup 0 reduces
// all of them, selects and publishes the selection record); workgroups [nrat, nrat + nprow) are the
// pivot-row workgroups, which wait for the record, replay and push the owner's row and commit it.
// Workgroups are dispatched in index order, so the ratio workgroups never wait for a slot behind
// the pivot-row workgroups that wait for them.  LEAN: beside the form-21 pass (32 VGPRs; both
// bodies' LDS rings are the same size).
#define DLP_PX_RATIO_ARGS                                                                                       \
    double *__restrict__ T, int64_t ld, int64_t rows, int64_t rows_elig, int64_t ncols, int64_t nprice,         \
        int64_t row_first, int32_t *basis, PricePart *pp, int ntiles, DevState *st, double *__restrict__ C,     \
        int64_t ldc, double *__restrict__ Cc, int64_t ldcc, double *__restrict__ P, double *__restrict__ rhs,   \
        int32_t *__restrict__ nzc, int nrat, double tol_dj, double tol_piv, int pricing, dlp_pivot *log,         \
        int64_t log_cap, const double *__restrict__ Ccp, const double *__restrict__ Pp,                          \
        const double *__restrict__ Cp, int prev_seal, const XPeers *xp, uint32_t xseq, uint32_t *bcnt, int brb, \
        int bnt, const double *Tn, int xs, Cond cd
// (xs = 2, passed at launch: as a compile-time constant hipcc gave the LEAN instance 34 VGPRs, at
// run time 30 of the 32 the form-21 pass leaves per SIMD)
#define DLP_PX_BODIES(KM, LEAN_, LCH_, RP_, RS_, CD_)                                                               \
    if ((int)blockIdx.x < nrat) {                                                                                \
        ratio_defer_body<KM, false, LEAN_, LCH_, RP_>(T, ld, rows, rows_elig, ncols, row_first, basis, pp,       \
                                                     ntiles, st, C, ldc, Cc, ldcc, P, rhs, nzc, nullptr,          \
                                                     nullptr, 2, tol_dj, tol_piv, pricing, log, log_cap, nrat,    \
                                                     Ccp, Pp, prev_seal, xp, xseq, bcnt, brb, bnt, Tn, xs, xseq, CD_); \
        return;                                                                                                  \
    }                                                                                                            \
    prow_defer_body<LEAN_, RS_>(T, ld, rows, ncols, nprice, st, C, ldc, P, nullptr, pp,      \
                                tol_dj, log, log_cap, 0, Cp, Pp, prev_seal, xp, xseq, bcnt, brb, bnt, Tn, 1,     \
                                (int)blockIdx.x - nrat, 1, CD_)
template <int KMAX>
__global__ __launch_bounds__(256) void pivot_x_kernel(DLP_PX_RATIO_ARGS) {
    DLP_PX_BODIES(KMAX, false, 4, kRatioRingPairs, kProwRingSteps, cd);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(32))) void pivot_x_lean_kernel(DLP_PX_RATIO_ARGS) {
    // (no condensed build: its 32 VGPRs are full; launch_pivot_x refuses a condensed session here)
    DLP_PX_BODIES(128, true, 0, kRatioRingPairs, kProwRingSteps, Cond{});
}
// The chain on CUs of its own (round 6): the grouped-ring selection with ROWS rows per wave (256 lanes
// cover the session's rthreads = 4 ROWS rows, so the exchange's candidate slots are unchanged) and the
// register pivot-row kernel, no VGPR budget; every workgroup resident (the caller's chain CUs hold two
// each at the ring's 64 KB)
template <int ROWS>
__global__ __launch_bounds__(256) void pivot_x_ring_kernel(DLP_PX_RATIO_ARGS) {
    if ((int)blockIdx.x < nrat) {
        ratio_defer_body<128, false, true, 0, 16, false, ROWS, 4>(
            T, ld, rows, rows_elig, ncols, row_first, basis, pp, ntiles, st, C, ldc, Cc, ldcc, P, rhs, nzc, nullptr,
            nullptr, 2, tol_dj, tol_piv, pricing, log, log_cap, nrat, Ccp, Pp, prev_seal, xp, xseq, bcnt, brb, bnt, Tn,
            xs, xseq, cd);
        return;
    }
    prow_defer_body<false>(T, ld, rows, ncols, nprice, st, C, ldc, P, nullptr, pp, tol_dj, log, log_cap, 0, Cp, Pp,
                           prev_seal, xp, xseq, bcnt, brb, bnt, Tn, 1, (int)blockIdx.x - nrat, 1, cd);
}
#undef DLP_PX_BODIES

// Multi-rank: P[s] from the exchanged bits, then the objective row + pricing.
__global__ __launch_bounds__(256) void commit_defer_kernel(
    double* __restrict__ T, int64_t ld, int64_t rows, int64_t ncols, int64_t nprice,
    DevState* st, const double* __restrict__ C, int64_t ldc, double* __restrict__ P,
    const int64_t* __restrict__ bits, PricePart* pp, double tol_dj, dlp_pivot* log,
    int64_t log_cap, const XPeers* xp, uint32_t xseq, Cond cd) {
    __shared__ PricePart lds_pp[4];
    __shared__ int s_ok;
    if (st->status != DLP_RUNNING) return;
    const int64_t slot = st->npivots - 1;
    if (blockIdx.x == 0) CHAIN_STAMP(slot, 12);
    const int s = st->blk - 1;
    const int64_t j = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2;
    d2 pr;
    pr.x = 0.0;
    pr.y = 0.0;
    if (xp) {   // peer exchange: this chunk's flag, then the row from this rank's region
        if (threadIdx.x == 0) s_ok = x_wait(xp, x_rflag(xp, xp->me, blockIdx.x), xseq) ? 1 : 0;
        __syncthreads();
        if (blockIdx.x == 0) CHAIN_STAMP(slot, 13);
        if (!s_ok) {
            if (threadIdx.x == 0) st->status = kStatusXFail;
            return;
        }
        if (j < ld) {
            uint64_t a = 0, b = 0;
            x_read_row_pair(xp, j, &a, &b);
            pr.x = __builtin_bit_cast(double, a);
            pr.y = __builtin_bit_cast(double, b);
        }
    } else if (j < ld) {
        pr = *(const d2*)(bits + j);
    }
    commit_row(T, ld, rows, ncols, nprice, st->npivots - 1, C, ldc, P, s, j, pr, pp, (int)blockIdx.x, tol_dj, log,
               log_cap, lds_pp, d2{0.0, 0.0}, 0.0, cd, cd.on ? st->sq : -1, cd.on ? st->bser : 0);
    if (blockIdx.x == 0) CHAIN_STAMP(slot, 14);
}

// Single rank: ratio test, selection and pivot row in ONE launch (saves a kernel
// boundary per pivot, and the pivot-row workgroups load the block's P rows while
// the ratio phase runs).  Blocks [0, nrat) run ratio_defer_body; blocks
// [nrat, nrat + nprow) are pivot-row workgroups, one 512-column tile each, which
// wait for st->go (bounded spin: a stall turns into DLP_ERR_HIP, never a hang),
// then replay T0[p] exactly as prow_defer_kernel and commit it (commit_row, with
// z_q from st->zq).  The last pivot-row workgroup to finish resets go and its
// ticket for the next launch.  Every block of the grid is resident at once
// (<= 2 * 129 workgroups of 256 threads at C3 against 8 per CU), and blocks are
// dispatched in index order, so the ratio blocks always run.
template <int KMAX>
__global__ __launch_bounds__(256) void pivot_defer_kernel(
    double* __restrict__ T, int64_t ld, int64_t rows, int64_t rows_elig, int64_t ncols,
    int64_t nprice, int64_t row_first, int32_t* basis, PricePart* pp, int ntiles, DevState* st,
    double* __restrict__ C, int64_t ldc, double* __restrict__ Cc, int64_t ldcc,
    double* __restrict__ P, double* __restrict__ rhs, int32_t* __restrict__ nzc, Cand* partials,
    int nrat, double tol_dj, double tol_piv, int pricing, dlp_pivot* log, int64_t log_cap) {
    if ((int)blockIdx.x < nrat) {
        ratio_defer_body<KMAX, true>(T, ld, rows, rows_elig, ncols, row_first, basis, pp, ntiles, st,
                                     C, ldc, Cc, ldcc, P, rhs, nzc, partials, nullptr, 1, tol_dj,
                                     tol_piv, pricing, log, log_cap, nrat);
        return;
    }
    __shared__ PricePart lds_pp[4];
    __shared__ double s_cp[KMAX];
    __shared__ int32_t s_pl[KMAX];
    __shared__ int s_ok;
    if (st->status != DLP_RUNNING) return;   // the same answer in every block of this launch
    const int tile = (int)blockIdx.x - nrat;
    const int64_t j = ((int64_t)tile * blockDim.x + threadIdx.x) * 2;
    const int64_t jc = j < ld ? j : ld - 2;
    // the block's earlier pivot rows at this lane's columns, before the wait (blk may
    // already be one past them if this block starts late: that row is not used)
    const int s0 = min(st->blk, KMAX);
    d2 pv[KMAX];
#pragma unroll
    for (int l = 0; l < KMAX; ++l)
        if (l < s0) pv[l] = *(const d2*)(P + (int64_t)l * ld + jc);
    if (threadIdx.x == 0) {
        int ok = 0;
        for (int it = 0; it < (1 << 24); ++it) {
            if (__hip_atomic_load(&st->go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                ok = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        s_ok = ok;
    }
    __syncthreads();
    const bool run = s_ok && st->status == DLP_RUNNING;
    if (!s_ok && threadIdx.x == 0) st->status = DLP_ERR_HIP;
    if (run) {
        const int s = st->blk - 1;
        const int32_t pl = st->p_local;
        for (int l = threadIdx.x; l < s; l += blockDim.x) {
            s_cp[l] = C[(int64_t)pl * ldc + l];
            s_pl[l] = st->pl[l];
        }
        __syncthreads();
        d2 pr;
        pr.x = 0.0;
        pr.y = 0.0;
        if (j < ld) {
            d2 t = *(const d2*)(T + (int64_t)pl * ld + j);
#pragma unroll
            for (int l = 0; l < KMAX; ++l) {
                if (l < s) {
                    const d2 v = l < s0 ? pv[l] : *(const d2*)(P + (int64_t)l * ld + j);
                    if (pl == s_pl[l]) {
                        t = v;
                    } else if (s_cp[l] != 0.0) {
                        t.x = __builtin_fma(-s_cp[l], v.x, t.x);
                        t.y = __builtin_fma(-s_cp[l], v.y, t.y);
                    }
                }
            }
            const double piv = st->piv;
            pr.x = t.x / piv;
            pr.y = t.y / piv;
        }
        // commit_row with z_q from the state (C[rows][s] is another block's store)
        const int64_t width = (ncols + 16) & ~(int64_t)15;
        if (j < ld) {
            *(d2*)(P + (int64_t)s * ld + j) = pr;
            if (s == 0)   // block start: pivot rows 1..K-1 := +0 (commit_row)
                for (int64_t l = 1; l < ldc; ++l) *(d2*)(P + l * ld + j) = d2{0.0, 0.0};
        }
        const double zq = st->zq;
        PricePart acc = pp_empty();
        if (j < width) {
            double* zp = T + rows * ld + j;
            d2 z = *(const d2*)zp;
            if (zq != 0.0) {
                z.x = __builtin_fma(-zq, pr.x, z.x);
                z.y = __builtin_fma(-zq, pr.y, z.y);
                *(d2*)zp = z;
            }
            price_pair(acc, z.x, z.y, j, nprice, tol_dj);
            if (log && j <= ncols && ncols < j + 2) {
                const int64_t k = st->npivots - 1;
                if (k >= 0 && k < log_cap) log[k].objective = (ncols == j) ? z.x : z.y;
            }
        }
        acc = block_price(acc, lds_pp);
        if (threadIdx.x == 0) pp[tile] = acc;
    }
    // the last pivot-row block to finish re-arms the flag for the next launch
    if (threadIdx.x == 0) {
        const int nprow = (int)gridDim.x - nrat;
        const unsigned prev =
            __hip_atomic_fetch_add(&st->ticket2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == (unsigned)nprow - 1) {
            __hip_atomic_store(&st->go, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&st->ticket2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// The tableau pass.  Workgroup (tile, band): 512 columns (2 doubles per lane,
// one 16-B access) of rb constraint rows.  Each lane holds P[0..kb)[its two
// columns] in registers for the whole band.  The band's coefficients C[i][l]
// (row-major, one contiguous rb*K block) are staged in LDS, negated, and one
// lane per row classifies its row once:
//   kUntouched  every C[i][l] == 0 and never a pivot row -> no load, no store
//   kDense      every step touches it                   -> branch-free fma chain
//   kSparse     some steps skip it                      -> fma + select per step
//   >= 0        last step at which it was the pivot row  -> start from P[that step]
// Per element the operations are exactly the eager sequence.
constexpr int kUntouched = -3, kDense = -2, kSparse = -1;

template <int K>
__device__ inline d2 chain_dense(d2 t, const d2* pr, const double* nf) {
#pragma unroll
    for (int l = 0; l < K; ++l) {
        t.x = __builtin_fma(nf[l], pr[l].x, t.x);
        t.y = __builtin_fma(nf[l], pr[l].y, t.y);
    }
    return t;
}

template <bool NT, int K>
__global__ __launch_bounds__(256) void pass_kernel(double* __restrict__ T, int64_t ld, int64_t rows,
                                                   int64_t width, const DevState* st,
                                                   const double* __restrict__ C, int64_t ldc,
                                                   const double* __restrict__ P, int rb) {
    extern __shared__ double lds[];   // nf[rb][K] (negated C), then int32 cls[rb]
    __shared__ int32_t s_pl[K];
    const int kb = st->blk;
    if (kb == 0) return;
    const int64_t j = (int64_t)blockIdx.x * kDeferTile + threadIdx.x * 2;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - 2;
    d2 pr[K];
#pragma unroll
    for (int l = 0; l < K; ++l) {
        pr[l].x = 0.0;
        pr[l].y = 0.0;
        if (l < kb) pr[l] = *(const d2*)(P + (int64_t)l * ld + jc);
    }
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    double* nf = lds;
    int32_t* cls = (int32_t*)(lds + (size_t)rb * K);
    const double* Cb = C + i0 * ldc;   // the band's rows: one contiguous block when ldc == K
    for (int idx = threadIdx.x; idx < nr * K; idx += blockDim.x) {
        const int r = idx / K, l = idx - r * K;
        nf[idx] = l < kb ? -Cb[(int64_t)r * ldc + l] : 0.0;
    }
    if (threadIdx.x < K) s_pl[threadIdx.x] = threadIdx.x < kb ? st->pl[threadIdx.x] : -1;
    __syncthreads();
    for (int r = threadIdx.x; r < nr; r += blockDim.x) {
        int last = -1, nz = 0;
        for (int l = 0; l < kb; ++l) {
            if (s_pl[l] == (int32_t)(i0 + r)) last = l;
            nz += nf[r * K + l] != 0.0;
        }
        cls[r] = last >= 0 ? last : (nz == kb ? kDense : (nz == 0 ? kUntouched : kSparse));
    }
    __syncthreads();
    const bool full = kb == K;
    for (int r = 0; r < nr; ++r) {
        const int c = cls[r];   // wave-uniform
        if (c == kUntouched) continue;
        double* row = T + (i0 + r) * ld;
        const double* f = nf + r * K;
        d2 t;
        if (c == kDense && full) {
            t = chain_dense<K>(ldv<NT>(row + jc), pr, f);
        } else {
            if (c >= 0) {
                t.x = 0.0;
                t.y = 0.0;
            } else {
                t = ldv<NT>(row + jc);
            }
#pragma unroll
            for (int l = 0; l < K; ++l) {
                if (l < kb && l >= c) {   // c < 0: every step; c >= 0: from the last pivot step on
                    if (l == c) {
                        t = pr[l];
                    } else {
                        d2 u;
                        u.x = __builtin_fma(f[l], pr[l].x, t.x);
                        u.y = __builtin_fma(f[l], pr[l].y, t.y);
                        const bool skip = f[l] == 0.0;
                        t.x = skip ? t.x : u.x;
                        t.y = skip ? t.y : u.y;
                    }
                }
            }
        }
        if (colok) stv<NT>(row + j, t);
    }
}

// Narrow form of the pass: one double per lane (256 columns per workgroup),
// so P[0..K) needs half the registers, and U rows per iteration, so each lane
// runs U independent fma chains (the chain, not HBM, limits the wide form at
// large K).  Dense groups (all U rows touched by every step, full block) take
// the branch-free path; everything else goes row by row through the generic
// replay.  Same per-element operations as pass_kernel.
template <bool NT, int K, int U>
__global__ __launch_bounds__(256) void pass1_kernel(double* __restrict__ T, int64_t ld, int64_t rows,
                                                    int64_t width, const DevState* st,
                                                    const double* __restrict__ C, int64_t ldc,
                                                    const double* __restrict__ P, int rb) {
    extern __shared__ double lds[];   // nf[rb][K] (negated C), then int32 cls[rb]
    __shared__ int32_t s_pl[K];
    const int kb = st->blk;
    if (kb == 0) return;
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - 1;
    double pr[K];
#pragma unroll
    for (int l = 0; l < K; ++l) pr[l] = (l < kb) ? P[(int64_t)l * ld + jc] : 0.0;
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    double* nf = lds;
    int32_t* cls = (int32_t*)(lds + (size_t)rb * K);
    const double* Cb = C + i0 * ldc;
    for (int idx = threadIdx.x; idx < nr * K; idx += blockDim.x) {
        const int r = idx / K, l = idx - r * K;
        nf[idx] = l < kb ? -Cb[(int64_t)r * ldc + l] : 0.0;
    }
    if (threadIdx.x < K) s_pl[threadIdx.x] = threadIdx.x < kb ? st->pl[threadIdx.x] : -1;
    __syncthreads();
    for (int r = threadIdx.x; r < nr; r += blockDim.x) {
        int last = -1, nz = 0;
        for (int l = 0; l < kb; ++l) {
            if (s_pl[l] == (int32_t)(i0 + r)) last = l;
            nz += nf[r * K + l] != 0.0;
        }
        cls[r] = last >= 0 ? last : (nz == kb ? kDense : (nz == 0 ? kUntouched : kSparse));
    }
    __syncthreads();
    const bool full = kb == K;
    int r = 0;
    if (full)
        for (; r + U <= nr; r += U) {
            bool dense = true;
#pragma unroll
            for (int u = 0; u < U; ++u) dense = dense && cls[r + u] == kDense;
            if (!dense) break;
            double t[U];
#pragma unroll
            for (int u = 0; u < U; ++u) t[u] = ldv1<NT>(T + (i0 + r + u) * ld + jc);
            const double* f = nf + r * K;
#pragma unroll
            for (int l = 0; l < K; l += 2) {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const d2 c = *(const d2*)(f + u * K + l);   // one 16-B LDS broadcast
                    t[u] = __builtin_fma(c.x, pr[l], t[u]);
                    t[u] = __builtin_fma(c.y, pr[l + 1], t[u]);
                }
            }
            if (colok)
#pragma unroll
                for (int u = 0; u < U; ++u) stv1<NT>(T + (i0 + r + u) * ld + j, t[u]);
        }
    for (; r < nr; ++r) {   // generic replay, one row at a time
        const int c = cls[r];
        if (c == kUntouched) continue;
        double* row = T + (i0 + r) * ld;
        const double* f = nf + r * K;
        double t = c >= 0 ? 0.0 : ldv1<NT>(row + jc);
#pragma unroll
        for (int l = 0; l < K; ++l) {
            if (l < kb && l >= c) {
                if (l == c) {
                    t = pr[l];
                } else {
                    const double u = __builtin_fma(f[l], pr[l], t);
                    t = f[l] == 0.0 ? t : u;
                }
            }
        }
        if (colok) stv1<NT>(row + j, t);
    }
}

// Scalar-coefficient form of the pass (forms 3-5).  The coefficients C[i][l]
// of a row are the same for every lane, so they are read with scalar loads
// straight from the C block (uniform address, read-only in this kernel) and
// enter v_fma_f64 as an SGPR operand with the negate modifier: no LDS traffic
// per fma, which bounds the LDS-staged forms at large K (one LDS broadcast
// per one or two fmas).  V doubles per lane (256 V columns per workgroup), U
// rows per group, P[0..K) in VGPRs.  Row class: nzc[i] = number of nonzero
// C[i][l] in the block (kept by ratio_defer_kernel), and the block's last
// pivot step on the row.  Same per-element operations as pass_kernel.
template <bool NT, int V>
__device__ inline void ldrow(double (&t)[V], const double* p) {
    if constexpr (V == 2) {
        const d2 v = ldv<NT>(p);
        t[0] = v.x;
        t[1] = v.y;
    } else {
        t[0] = ldv1<NT>(p);
    }
}
template <bool NT, int V>
__device__ inline void strow(double* p, const double (&t)[V]) {
    if constexpr (V == 2) {
        d2 v;
        v.x = t[0];
        v.y = t[1];
        stv<NT>(p, v);
    } else {
        stv1<NT>(p, t[0]);
    }
}

// The block's coefficients are read-only during the pass: through the constant
// address space, wave-uniform loads of them are always scalar loads.
typedef __attribute__((address_space(4))) const double* cdptr;

// T: the tableau read; Tout: where the rows go (== T in place; lookahead: the other
// buffer, so untouched rows are copied and an empty block copies everything); bd: the
// block (DevState::blk / pl, or a sealed copy).
template <bool NT, int K, int V, int U, bool PART, bool DEEP = false>
__device__ __forceinline__ void pass_s_body(const double* __restrict__ T, double* __restrict__ Tout,
                                            int64_t ld, int64_t rows, int64_t width,
                                            const BlockDesc* __restrict__ bd,
                                            const double* __restrict__ C, int64_t ldc,
                                            const double* __restrict__ P,
                                            const int32_t* __restrict__ nzc, int rb, int tails) {
    __shared__ int32_t cls[1024];
    const int kb = bd->blk;
    const bool outplace = Tout != T;
    // tails (the session's K is this instance's K): the block's unused steps were zeroed at
    // its start (C and P tails: ratio kernel, commit_row), so the full-block instance runs
    // partial blocks too, as one launch.  Otherwise two launches per pass: the full-block
    // instance (kb == K) and the partial one (0 < kb < K: a window's last block, or one cut
    // short by termination; kb == 0 out of place: a copy), so that neither carries the
    // other's register pressure; exactly one of them runs
    if ((kb == 0 && !outplace) || (PART ? kb == K : (kb != K && !tails))) return;
    const int64_t j = (int64_t)blockIdx.x * (256 * V) + threadIdx.x * V;
    const bool colok = j < width;
    const int64_t jc = colok ? j : width - V;
    double pr[K][V];
#pragma unroll
    for (int l = 0; l < K; ++l) {
        double v[V];
        // rows l >= kb are not used (and need not exist: P holds d.K <= K rows)
        ldrow<false, V>(v, P + (int64_t)(l < kb ? l : 0) * ld + jc);
#pragma unroll
        for (int e = 0; e < V; ++e) pr[l][e] = l < kb ? v[e] : 0.0;
    }
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    for (int r = threadIdx.x; r < nr; r += blockDim.x) {
        const int nz = nzc[i0 + r];
        int last = -1;
        for (int l = 0; l < kb; ++l)
            if (bd->pl[l] == (int32_t)(i0 + r)) last = l;
        cls[r] = last >= 0 ? last : (nz == kb ? kDense : (nz == 0 ? kUntouched : kSparse));
    }
    __syncthreads();
    // dense groups: U rows, every step of the block touches every row.  The next dense
    // group's rows are loaded before this group's fma chains, so every wave keeps two
    // groups of HBM loads in flight (vector loads retire in order: vmcnt covers them,
    // while the coefficients' scalar loads wait on lgkmcnt only).
    auto dense_at = [&](int r0) {
        if (r0 + U > nr) return false;
        bool d = true;
#pragma unroll
        for (int u = 0; u < U; ++u) d = d && cls[r0 + u] == kDense;
        return d;
    };
    const double* cbase = C + i0 * ldc;
    // one dense group: t = rows r0..r0+U-1 (already loaded), all K steps, store.
    // Coefficients in chunks of LC steps x U rows (16 doubles = 32 SGPRs), double
    // buffered: scalar loads return out of order, so a chunk is waited for (lgkmcnt(0))
    // BEFORE the next chunk's loads are issued, and those then land while the current
    // chunk's fmas run.  sched_barriers keep the compiler from re-merging the two.
    constexpr int LC = (16 / U) < K ? (16 / U) : K;
    auto fetch = [&](double (&f)[U][LC], cdptr cb, int l0) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int l = 0; l < LC; ++l) f[u][l] = cb[u * ldc + l0 + l];
    };
    auto chain = [&](double (&t)[U][V], const double (&f)[U][LC], int l0) {
#pragma unroll
        for (int l = 0; l < LC; ++l)
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int e = 0; e < V; ++e)
                    t[u][e] = __builtin_fma(-f[u][l], pr[l0 + l][e], t[u][e]);
    };
    // a partial block runs the full-block code: chunks past step kb-1 are skipped, and in
    // the chunk holding it the coefficients of steps >= kb are zeroed (scalar selects).
    // With P[l] = +0 for l >= kb (above) such a step is fma(-(+0), +0, t) = t + (-0) = t
    // for every t, so the result is exactly that of the kb real steps.
    auto mask = [&](double (&f)[U][LC], int l0) {
        if constexpr (PART) {
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int l = 0; l < LC; ++l) f[u][l] = (l0 + l < kb) ? f[u][l] : 0.0;
        }
    };
    auto group = [&](double (&t)[U][V], int r0) {
        const cdptr cb = (cdptr)(cbase + (int64_t)r0 * ldc);
        {
            double fa[U][LC], fb[U][LC];
            fetch(fa, cb, 0);
#pragma unroll
            for (int l0 = 0; l0 < K; l0 += 2 * LC) {
                if (PART && l0 >= kb) break;
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): chunk fa has landed
                const bool nb = l0 + LC < K && (!PART || l0 + LC < kb);
                if (nb) fetch(fb, cb, l0 + LC);
                mask(fa, l0);
                __builtin_amdgcn_sched_barrier(0);
                chain(t, fa, l0);
                __builtin_amdgcn_sched_barrier(0);
                if (nb) {
                    __builtin_amdgcn_s_waitcnt(0xC07F);   // chunk fb has landed
                    if (l0 + 2 * LC < K && (!PART || l0 + 2 * LC < kb)) fetch(fa, cb, l0 + 2 * LC);
                    mask(fb, l0 + LC);
                    __builtin_amdgcn_sched_barrier(0);
                    chain(t, fb, l0 + LC);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        if (colok)
#pragma unroll
            for (int u = 0; u < U; ++u) strow<NT, V>(Tout + (i0 + r0 + u) * ld + j, t[u]);
    };
    auto load = [&](double (&t)[U][V], int r0) {
#pragma unroll
        for (int u = 0; u < U; ++u) ldrow<NT, V>(t[u], T + (i0 + r0 + u) * ld + jc);
    };
    double ta[U][V], tb[U][V];
    int r = 0;
    while (r < nr) {
        if (DEEP && dense_at(r)) {
            // form 20: three register buffers, so the rows of the next TWO dense groups
            // are in flight while one group's chains run
            double tc[U][V];
            load(ta, r);
            bool nb = dense_at(r + U);
            load(tb, nb ? r + U : r);
            while (true) {
                const bool nc = nb && dense_at(r + 2 * U);
                load(tc, nc ? r + 2 * U : r);
                __builtin_amdgcn_sched_barrier(0);
                group(ta, r);
                r += U;
                if (!nb) break;
                const bool nd = nc && dense_at(r + 2 * U);
                load(ta, nd ? r + 2 * U : r);
                __builtin_amdgcn_sched_barrier(0);
                group(tb, r);
                r += U;
                if (!nc) break;
                const bool ne = nd && dense_at(r + 2 * U);
                load(tb, ne ? r + 2 * U : r);
                __builtin_amdgcn_sched_barrier(0);
                group(tc, r);
                r += U;
                if (!nd) break;
                nb = ne;
            }
            continue;
        }
        if (dense_at(r)) {
            // a run of dense groups, ping-ponging two register buffers
            load(ta, r);
            // The prefetch is unconditional (at the end of a run it re-reads the current
            // group's rows, an L2 hit), so the in-order vmcnt wait for the group being
            // computed is the same on every path and leaves the prefetch in flight.
            while (true) {
                const bool nb = dense_at(r + U);
                load(tb, nb ? r + U : r);
                __builtin_amdgcn_sched_barrier(0);   // keep the prefetch ahead of the chains
                group(ta, r);
                r += U;
                if (!nb) break;
                const bool na = dense_at(r + U);
                load(ta, na ? r + U : r);
                __builtin_amdgcn_sched_barrier(0);
                group(tb, r);
                r += U;
                if (!na) break;
            }
            continue;
        }
        // generic replay, one row (sparse rows, the block's pivot rows, partial blocks): a
        // runtime loop over the steps with P[l] re-read from L2, so that the unrolled
        // register copy serves only the dense path
        const int c = cls[r];
        if (c == kUntouched && outplace) {
            double t[V];
            ldrow<NT, V>(t, T + (i0 + r) * ld + jc);
            if (colok) strow<NT, V>(Tout + (i0 + r) * ld + j, t);
        } else if (c != kUntouched) {
            const double* row = T + (i0 + r) * ld;
            const double* cr = C + (i0 + r) * ldc;
            double t[V];
            int l = 0;
            if (c >= 0) {
                ldrow<false, V>(t, P + (int64_t)c * ld + jc);
                l = c + 1;
            } else {
                ldrow<NT, V>(t, row + jc);
            }
            for (; l < kb; ++l) {
                const double f = cr[l];
                if (f != 0.0) {
                    double pv[V];
                    ldrow<false, V>(pv, P + (int64_t)l * ld + jc);
#pragma unroll
                    for (int e = 0; e < V; ++e) t[e] = __builtin_fma(-f, pv[e], t[e]);
                }
            }
            if (colok) strow<NT, V>(Tout + (i0 + r) * ld + j, t);
        }
        r += 1;
    }
}

template <bool NT, int K, int V, int U, bool PART, bool DEEP = false>
__global__ __launch_bounds__(256) void pass_s_kernel(const double* __restrict__ T, double* __restrict__ Tout,
                                                     int64_t ld, int64_t rows, int64_t width,
                                                     const BlockDesc* __restrict__ bd,
                                                     const double* __restrict__ C, int64_t ldc,
                                                     const double* __restrict__ P,
                                                     const int32_t* __restrict__ nzc, int rb, int tails) {
    pass_s_body<NT, K, V, U, PART, DEEP>(T, Tout, ld, rows, width, bd, C, ldc, P, nzc, rb, tails);
}

// The same body held to 3 waves per SIMD (<= 168 VGPRs; form 4 alone takes 170, which
// allocates 176 and leaves 2 waves per SIMD).
template <bool NT, int K, int V, int U, bool PART>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void pass_s3_kernel(
    const double* __restrict__ T, double* __restrict__ Tout, int64_t ld, int64_t rows, int64_t width,
    const BlockDesc* __restrict__ bd, const double* __restrict__ C, int64_t ldc,
    const double* __restrict__ P, const int32_t* __restrict__ nzc, int rb, int tails) {
    pass_s_body<NT, K, V, U, PART>(T, Tout, ld, rows, width, bd, C, ldc, P, nzc, rb, tails);
}

// Streamed form of the pass (forms 6-9): pass_s_body's per-element operations,
// with three changes aimed at the HBM stream.
//  * Work order.  A 1-D grid; workgroup b works on position q of a list of
//    (tile, band) pairs ordered by groups of kPassBands bands, tile-major inside
//    a group, and the list is cut into 8 equal contiguous pieces, piece b % 8
//    going to the workgroups that share b's XCD (blocks are dealt round-robin
//    over the 8 XCDs: MI355X_MICROARCH.md, workgroup dispatch).  So the
//    workgroups resident on one XCD at a time share a few tiles' P slices and a
//    few bands' coefficients in that XCD's L2, instead of every workgroup
//    fetching both again from the Infinity Cache.  Placement only moves speed.
//  * Dense groups first.  The band's dense groups (U rows, every step of the
//    block touches every row) are compacted into a list in LDS and streamed
//    through a ring of D register buffers: the rows of D-1 groups are in flight
//    while one group's fma chains run.  Everything else (sparse rows, the
//    block's pivot rows, rows of partly dense groups) follows, row by row,
//    through the generic replay.  Rows are independent, so order is free.
//  * Coefficients.  Scalar loads in chunks of LC steps x U rows, double
//    buffered, and the next dense group's first chunk is fetched during the
//    current group's last chunk (full blocks: K / LC is even).
constexpr int kPassBands = 16;   // bands per group of the work order

// Buffer access to one band of the tableau: the descriptor is built once from
// wave-uniform values, every lane keeps ONE 32-bit column offset, and the row
// offset is a scalar (soffset).  aux 2 = nt.
template <bool NT, int V>
__device__ inline void bld(double (&t)[V], __amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    if constexpr (V == 2) {
        const u4v x = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, soff, NT ? 2 : 0);
        const d2 v = __builtin_bit_cast(d2, x);
        t[0] = v.x;
        t[1] = v.y;
    } else {
        const u2v x = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, NT ? 2 : 0);
        t[0] = __builtin_bit_cast(double, x);
    }
}
template <bool NT, int V>
__device__ inline void bst(const double (&t)[V], __amdgpu_buffer_rsrc_t rs, int voff, int soff) {
    if constexpr (V == 2) {
        d2 v;
        v.x = t[0];
        v.y = t[1];
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), rs, voff, soff, NT ? 2 : 0);
    } else {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, t[0]), rs, voff, soff, NT ? 2 : 0);
    }
}

template <int K, int V, int U>
struct PassGeo {
    static constexpr int LC = (16 / U) < K ? (16 / U) : K;   // steps per coefficient chunk
    static constexpr int NCH = K / LC;                       // chunks per group
};

template <bool NT, int K, int V, int U, int D, bool PART>
__global__ __launch_bounds__(256) void pass_r_kernel(double* __restrict__ T, int64_t ld,
                                                     int64_t rows, int64_t width,
                                                     const DevState* __restrict__ st,
                                                     const double* __restrict__ C, int64_t ldc,
                                                     const double* __restrict__ P,
                                                     const int32_t* __restrict__ nzc, int rb,
                                                     int ntiles, int nbands, int order) {
    static_assert(PassGeo<K, V, U>::NCH % 2 == 0, "the cross-group prefetch needs an even chunk count");
    __shared__ int32_t cls[1024];
    __shared__ int16_t dgl[512];
    __shared__ int32_t s_wtot[4];
    const int kb = st->blk;
    if (kb == 0 || (PART ? kb == K : kb != K)) return;
    // (tile, band) of this workgroup: order 1 = the XCD work order above; order 0 =
    // tile-fastest over the whole grid (consecutive workgroups stream one row range)
    const int64_t total = (int64_t)ntiles * nbands;
    int tile, band;
    if (order) {
        const int64_t per = (total + 7) >> 3;
        const int64_t q = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
        if ((int64_t)(blockIdx.x >> 3) >= per || q >= total) return;
        const int bgrp = (int)(q / ((int64_t)kPassBands * ntiles));
        const int rr = (int)(q - (int64_t)bgrp * kPassBands * ntiles);
        const int nbg = min(kPassBands, nbands - bgrp * kPassBands);
        tile = rr / nbg;
        band = bgrp * kPassBands + rr % nbg;
    } else if (order == 2) {
        // XCD b % 8 owns a range of ceil(ntiles / 8) column tiles and walks it band by
        // band: its resident workgroups share those tiles' P slices in its L2, and the
        // 8 XCDs together sweep whole rows, as the eager update does
        const int t8 = (ntiles + 7) >> 3;
        const int x = blockIdx.x & 7, k = blockIdx.x >> 3;
        const int tx0 = x * t8, ntx = min(t8, ntiles - tx0);
        if (ntx <= 0 || k >= ntx * nbands) return;
        band = k / ntx;
        tile = tx0 + k % ntx;
    } else {
        if ((int64_t)blockIdx.x >= total) return;
        band = (int)(blockIdx.x / ntiles);
        tile = (int)(blockIdx.x - (int64_t)band * ntiles);
    }

    const int64_t j = (int64_t)tile * (256 * V) + threadIdx.x * V;
    const int64_t jc = j < width ? j : width - V;
    double pr[K][V];
#pragma unroll
    for (int l = 0; l < K; ++l) {
        double v[V];
        ldrow<false, V>(v, P + (int64_t)(l < kb ? l : 0) * ld + jc);
#pragma unroll
        for (int e = 0; e < V; ++e) pr[l][e] = l < kb ? v[e] : 0.0;
    }
    const int64_t i0 = (int64_t)band * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    for (int r = threadIdx.x; r < nr; r += blockDim.x) {
        const int nz = nzc[i0 + r];
        int last = -1;
        for (int l = 0; l < kb; ++l)
            if (st->pl[l] == (int32_t)(i0 + r)) last = l;
        cls[r] = last >= 0 ? last : (nz == kb ? kDense : (nz == 0 ? kUntouched : kSparse));
    }
    __syncthreads();
    // compact the dense groups into dgl[0..ndg); their rows leave the generic loop
    const int ng = nr / U;
    int ndg = 0;
    for (int base = 0; base < ng; base += 256) {
        const int g = base + (int)threadIdx.x;
        bool d = g < ng;
        if (d)
#pragma unroll
            for (int u = 0; u < U; ++u) d = d && cls[g * U + u] == kDense;
        const uint64_t m = __ballot(d);
        const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
        const int pre = __popcll(m & ((1ull << ln) - 1ull));
        if (ln == 0) s_wtot[wv] = __popcll(m);
        __syncthreads();
        int off = ndg;
        for (int w = 0; w < wv; ++w) off += s_wtot[w];
        if (d) {
            dgl[off + pre] = (int16_t)g;
#pragma unroll
            for (int u = 0; u < U; ++u) cls[g * U + u] = kUntouched;
        }
        ndg += s_wtot[0] + s_wtot[1] + s_wtot[2] + s_wtot[3];
        __syncthreads();
    }

    constexpr int LC = PassGeo<K, V, U>::LC;
    constexpr int NCH = PassGeo<K, V, U>::NCH;
    const double* cbase = C + i0 * ldc;
    auto fetch = [&](double (&f)[U][LC], cdptr cb, int l0) {
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int l = 0; l < LC; ++l) f[u][l] = cb[u * ldc + l0 + l];
    };
    auto chain = [&](double (&t)[U][V], const double (&f)[U][LC], int l0) {
#pragma unroll
        for (int l = 0; l < LC; ++l)
#pragma unroll
            for (int u = 0; u < U; ++u)
#pragma unroll
                for (int e = 0; e < V; ++e)
                    t[u][e] = __builtin_fma(-f[u][l], pr[l0 + l][e], t[u][e]);
    };
    // the chunk holding step kb-1: a uniform branch per step (no per-element selects)
    auto chain_part = [&](double (&t)[U][V], const double (&f)[U][LC], int l0) {
#pragma unroll
        for (int l = 0; l < LC; ++l)
            if (l0 + l < kb)
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int e = 0; e < V; ++e)
                        t[u][e] = __builtin_fma(-f[u][l], pr[l0 + l][e], t[u][e]);
    };
    auto grow = [&](int g) { return (int)__builtin_amdgcn_readfirstlane(dgl[g]) * U; };
    // the band through one buffer descriptor (the launcher keeps rb * ld * 8 < 2^31).
    // Lanes past the last column work on (and store) the last column group: the
    // same operations on the same inputs give the same bits as its owner lane, so
    // every store is unconditional (no exec-masked stores for vmcnt to second-guess)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(T + i0 * ld), (short)0, (int)((int64_t)nr * ld * 8), 0x00020000);
    const int voff = (int)(jc * 8);
    const int ld8 = (int)(ld * 8);
    auto load = [&](double (&t)[U][V], int r0) {
#pragma unroll
        for (int u = 0; u < U; ++u) bld<NT, V>(t[u], rs, voff, (r0 + u) * ld8);
    };
    auto store = [&](const double (&t)[U][V], int r0) {
#pragma unroll
        for (int u = 0; u < U; ++u) bst<NT, V>(t[u], rs, voff, (r0 + u) * ld8);
    };
    double fa[U][LC], fb[U][LC];
    // full block: fa holds chunk 0 of this group on entry and chunk 0 of group rn on exit
    auto group_full = [&](double (&t)[U][V], int r0, int rn) {
        const cdptr cb = (cdptr)(cbase + (int64_t)r0 * ldc);
        const cdptr cn = (cdptr)(cbase + (int64_t)rn * ldc);
#pragma unroll
        for (int c = 0; c < NCH; c += 2) {
            __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): fa has landed
            fetch(fb, cb, (c + 1) * LC);
            __builtin_amdgcn_sched_barrier(0);
            chain(t, fa, c * LC);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_waitcnt(0xC07F);   // fb has landed
            if (c + 2 < NCH)
                fetch(fa, cb, (c + 2) * LC);
            else
                fetch(fa, cn, 0);
            __builtin_amdgcn_sched_barrier(0);
            chain(t, fb, (c + 1) * LC);
            __builtin_amdgcn_sched_barrier(0);
        }
        store(t, r0);
    };
    // partial block: chunks up to step kb-1, the last one masked
    auto group_part = [&](double (&t)[U][V], int r0) {
        const cdptr cb = (cdptr)(cbase + (int64_t)r0 * ldc);
        fetch(fa, cb, 0);
#pragma unroll
        for (int c = 0; c < NCH; c += 2) {
            if (c * LC < kb) {
                __builtin_amdgcn_s_waitcnt(0xC07F);
                if ((c + 1) * LC < kb) fetch(fb, cb, (c + 1) * LC);
                __builtin_amdgcn_sched_barrier(0);
                if ((c + 1) * LC <= kb)
                    chain(t, fa, c * LC);
                else
                    chain_part(t, fa, c * LC);
                __builtin_amdgcn_sched_barrier(0);
                if ((c + 1) * LC < kb) {
                    __builtin_amdgcn_s_waitcnt(0xC07F);
                    if ((c + 2) * LC < kb && c + 2 < NCH) fetch(fa, cb, (c + 2) * LC);
                    __builtin_amdgcn_sched_barrier(0);
                    if ((c + 2) * LC <= kb)
                        chain(t, fb, (c + 1) * LC);
                    else
                        chain_part(t, fb, (c + 1) * LC);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
        }
        store(t, r0);
    };

    if (ndg > 0) {
        double buf[D][U][V];
#pragma unroll
        for (int b = 0; b < D - 1; ++b) load(buf[b], grow(b < ndg ? b : ndg - 1));
        if constexpr (!PART) fetch(fa, (cdptr)(cbase + (int64_t)grow(0) * ldc), 0);
        for (int g0 = 0; g0 < ndg; g0 += D) {
#pragma unroll
            for (int b = 0; b < D; ++b) {
                const int gi = g0 + b;
                if (gi < ndg) {
                    // the ring's next group: rows D-1 groups ahead (clamped: an L2 hit)
                    const int ga = gi + D - 1 < ndg ? gi + D - 1 : ndg - 1;
                    load(buf[(b + D - 1) % D], grow(ga));
                    __builtin_amdgcn_sched_barrier(0);
                    if constexpr (!PART)
                        group_full(buf[b], grow(gi), grow(gi + 1 < ndg ? gi + 1 : gi));
                    else
                        group_part(buf[b], grow(gi));
                }
            }
        }
    }
    // everything else, row by row (as pass_s_body's generic replay)
    for (int r = 0; r < nr; ++r) {
        const int c = cls[r];
        if (c == kUntouched) continue;
        const double* cr = C + (i0 + r) * ldc;
        double t[V];
        int l = 0;
        if (c >= 0) {
            ldrow<false, V>(t, P + (int64_t)c * ld + jc);
            l = c + 1;
        } else {
            bld<NT, V>(t, rs, voff, r * ld8);
        }
        for (; l < kb; ++l) {
            const double f = cr[l];
            if (f != 0.0) {
                double pv[V];
                ldrow<false, V>(pv, P + (int64_t)l * ld + jc);
#pragma unroll
                for (int e = 0; e < V; ++e) t[e] = __builtin_fma(-f, pv[e], t[e]);
            }
        }
        bst<NT, V>(t, rs, voff, r * ld8);
    }
}


// Row classes of a band (pass_s_body's rule) for the 64-step passes: every row from nzc,
// then each step's pivot row raised to the step index (LDS atomic max: the last step that
// pivoted on the row wins; steps >= 0 exceed every class code).  One load per thread
// instead of a scan of the step table per row.  The caller syncs.
__device__ inline void classify_band(int32_t* cls, const BlockDesc* __restrict__ bd,
                                     const int32_t* __restrict__ nzc, int64_t i0, int nr, int kb) {
    for (int r = threadIdx.x; r < nr; r += blockDim.x) {
        const int nz = nzc[i0 + r];
        cls[r] = nz == kb ? kDense : (nz == 0 ? kUntouched : kSparse);
    }
    __syncthreads();
    for (int l = threadIdx.x; l < kb; l += blockDim.x) {
        const int64_t r = (int64_t)bd->pl[l] - i0;
        if (bd->pl[l] >= 0 && r >= 0 && r < nr) atomicMax(&cls[r], l);
    }
}

// Form 21: the pass at K = 64 with the coefficients broadcast by DPP.  At 64 steps per
// element the scalar coefficient path of forms 3-5 stalls: every chunk of 2 rows x 8
// steps is a scalar load that misses to L2 (~800 cycles under the stream) against ~128
// cycles of fmas, and a pass took 16 ms where the same chain with no coefficient loads
// takes 7.1 (tools/passlab.hip, profiles/r02j/).  Here the coefficients travel as
// ordinary vector loads, well ahead of use: lane n of each 16-lane row loads steps
// (2n, 2n+1) of a 32-step half of its row's coefficient row with one 16-B load, and
// v_fmac_f64_dpp ... row_newbcast:n reads lane n's value for the whole row, so the fma
// takes its coefficient straight from another lane's register (neg modifier: fma(-c, p, t),
// the eager operation).  1 double x 2 rows per lane, P[0..64) in 128 VGPRs, buffer
// accesses with one 32-bit column offset per lane: 166 VGPRs, 3 waves per SIMD.
// Coefficient registers are written only by loads (no VALU write within two
// instructions of a DPP read: tests/test_isa.py audits the built code object).  Partial
// blocks run the same code: their unused steps were zeroed at block start (C and P tails).
template <int N>
__device__ __forceinline__ void fmac_bc(double& t, double c, double p) {
    asm("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(t)
        : "v"(c), "v"(p), "n"(N));
}
template <int N>
__device__ __forceinline__ double bc_mov(double v) {
    return __builtin_amdgcn_update_dpp(0.0, v, 0x150 + N, 0xf, 0xf, false);
}
// step l of both rows: half h = l / 32, (even, odd) register e = l & 1, lane (l & 31) / 2
template <int L>
__device__ __forceinline__ void dpp_step(double (&t)[2], const double (&c)[2][2][2], const double (&pr)[64]) {
    constexpr int h = L / 32, e = L & 1, n = (L & 31) >> 1;
    fmac_bc<n>(t[0], c[0][h][e], pr[L]);
    fmac_bc<n>(t[1], c[1][h][e], pr[L]);
}
template <int L0, int... I>
__device__ __forceinline__ void dpp_half(double (&t)[2], const double (&c)[2][2][2], const double (&pr)[64],
                                         std::integer_sequence<int, I...>) {
    (dpp_step<L0 + I>(t, c, pr), ...);
}

// Generic replay of one row of class cl (a pivot row at step cl >= 0: start from P[cl]; a
// sparse row: skip the steps whose coefficient is 0) over the 64 steps, P[0..64) of the
// lane's column in registers (unrolled: no dynamic register index), the row's coefficients
// from f(l) (uniform).  The tails of a partial block have f == 0 and are skipped.
template <typename F>
__device__ __forceinline__ double replay_row(double t, int cl, const double (&pr)[64], F f) {
#pragma unroll
    for (int l = 0; l < 64; ++l) {
        const double c = f(l);
        if (l == cl)
            t = pr[l];
        else if (l > cl && c != 0.0)
            t = __builtin_fma(-c, pr[l], t);
    }
    return t;
}

// PUB (lookahead): the output rows are stored write-through (sc1) and every workgroup, once
// all its waves have drained their stores, adds 1 to its band's count, so the next block's
// selections can read a finished band from Tout instead of replaying this block on it
// (band_done; MI355X_MICROARCH.md, inter-workgroup visibility, first row of the sc1 table).
template <bool NT, bool PUB = false>
__global__ __launch_bounds__(256) void pass_d_kernel(const double* __restrict__ T, double* __restrict__ Tout,
                                                     int64_t ld, int64_t rows, int64_t width,
                                                     const BlockDesc* __restrict__ bd,
                                                     const double* __restrict__ C, int64_t ldc,
                                                     const double* __restrict__ P,
                                                     const int32_t* __restrict__ nzc, int rb,
                                                     uint32_t* bcnt = nullptr) {
    constexpr int K = 64, U = 2;
    constexpr int kSt = (NT ? 2 : 0) | (PUB ? kAuxSc1 : 0);   // store policy
    __shared__ int32_t cls[1024];
    const int kb = bd->blk;
    const bool outplace = Tout != T;
    if (kb == 0 && !outplace) return;   // full and partial blocks alike (zeroed tails)
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool colok = j < width;
    const int jc = (int)(colok ? j : width - 1);
    double pr[K];   // all 64 rows: a partial block's P[l >= kb] is +0 (zeroed at block start)
#pragma unroll
    for (int l = 0; l < K; ++l) pr[l] = P[(int64_t)l * ld + jc];
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    classify_band(cls, bd, nzc, i0, nr, kb);
    __syncthreads();
    // band descriptors (the caller keeps rb * ld * 8 < 2^31): rows at soffset r * ld8;
    // stores of lanes past the width go out of range and are dropped
    const int ld8 = (int)(ld * 8);
    const __amdgpu_buffer_rsrc_t rt = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(T + i0 * ld), (short)0, (int)((int64_t)nr * ld * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Tout + i0 * ld), (short)0, (int)((int64_t)nr * ld * 8), 0x00020000);
    const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(C + i0 * ldc), (short)0, (int)((int64_t)nr * ldc * 8), 0x00020000);
    const int voff = jc * 8;
    const int soff_bad = 0x7fffff00;
    const int voff_st = colok ? voff : soff_bad;
    const int coff = (threadIdx.x & 15) * 16;
    auto dense_at = [&](int r0) {
        if (r0 + U > nr) return false;
        return cls[r0] == kDense && cls[r0 + 1] == kDense;
    };
    double c[U][2][2];   // [row][half][even/odd step]
    auto loadc = [&](int r0, int h) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u4v x = __builtin_amdgcn_raw_buffer_load_b128(rc, coff + h * 256, (r0 + u) * (int)ldc * 8, 0);
            const d2 v = __builtin_bit_cast(d2, x);
            c[u][h][0] = v.x;
            c[u][h][1] = v.y;
        }
    };
    auto loadt = [&](double (&t)[U], int r0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u2v x = __builtin_amdgcn_raw_buffer_load_b64(rt, voff, (r0 + u) * ld8, NT ? 2 : 0);
            t[u] = __builtin_bit_cast(double, x);
        }
    };
    // one dense group (rows r0, r0+1 in t; their coefficients in c), with the loads of the
    // next group rn issued in vmcnt order: its rows first, the first half of its
    // coefficients once this group's first half has run, the second half at the end
    auto group = [&](double (&t)[U], double (&tn)[U], int r0, int rn) {
        loadt(tn, rn);
        __builtin_amdgcn_sched_barrier(0);
        dpp_half<0>(t, c, pr, std::make_integer_sequence<int, 32>{});
        __builtin_amdgcn_sched_barrier(0);
        loadc(rn, 0);
        __builtin_amdgcn_sched_barrier(0);
        dpp_half<32>(t, c, pr, std::make_integer_sequence<int, 32>{});
        __builtin_amdgcn_sched_barrier(0);
        loadc(rn, 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, t[u]), ro, voff_st, (r0 + u) * ld8,
                                                  kSt);
    };
    double ta[U], tb[U];
    int r = 0;
    while (r < nr) {
        if (dense_at(r)) {
            // a run of dense groups (the next group's loads are clamped to the current
            // one at the end of a run: harmless re-reads)
            loadt(ta, r);
            loadc(r, 0);
            loadc(r, 1);
            while (true) {
                const bool nb = dense_at(r + U);
                group(ta, tb, r, nb ? r + U : r);
                r += U;
                if (!nb) break;
                const bool na = dense_at(r + U);
                group(tb, ta, r, na ? r + U : r);
                r += U;
                if (!na) break;
            }
            continue;
        }
        // generic replay, one row (as pass_s_body)
        const int cl = cls[r];
        if (cl == kUntouched && outplace) {
            const u2v x = __builtin_amdgcn_raw_buffer_load_b64(rt, voff, r * ld8, NT ? 2 : 0);
            __builtin_amdgcn_raw_buffer_store_b64(x, ro, voff_st, r * ld8, kSt);
        } else if (cl != kUntouched) {
            const double* cr = C + (i0 + r) * ldc;
            double t = 0.0;
            if (cl < 0)
                t = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rt, voff, r * ld8, NT ? 2 : 0));
            t = replay_row(t, cl, pr, [&](int l) { return cr[l]; });
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, t), ro, voff_st, r * ld8, kSt);
        }
        r += 1;
    }
    if constexpr (PUB) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its sc1 stores are through
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(&bcnt[blockIdx.y], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// Form 23: form 21's arithmetic (P[0..64) of one column per lane in 128 VGPRs, the
// coefficients broadcast by v_fmac_f64_dpp) with the tableau rows and their coefficient
// rows staged through an LDS ring instead of registers.  Form 21 holds one 2-row group
// ahead in registers: 1 KB in flight per wave, so the stream is latency-bound (4.2 TB/s).
// Here each wave keeps D groups of U rows in flight by LDS-DMA (global_load_lds_dwordx4:
// no VGPRs): ring slot = U rows x the wave's 64 columns, then the U rows' 64 coefficients
// (DMA k: rows 2k, 2k+1, lane l's 16 B = row 2k + l / 32, columns / steps 2 (l % 32), +1).
// The DMAs are issued from inline asm so that hipcc does not count them (it would wait
// vmcnt(0) before the next LDS read, draining the ring: cdna_hip_programming.md, glds);
// the kernel waits with its own counted vmcnt, which relies on every group issuing exactly
// U DMAs and U stores (rows with nothing to store aim a store out of range).  Groups whose
// U rows are all dense run the chains from LDS; any other group replays row by row
// (replay_row: T and the coefficients from the slot, P from the registers).  Lab:
// 7.3-7.5 ms per C3 pass against form 21's 8.2-8.5 (tools/passlab.hip f4r, bit-exact).
// newer than group g's U DMAs: U per prologue group still to come and 2 U (U stores + U
// DMAs) per finished group: U (D - 1) + U g while g < D - 1, then 2 U (D - 1)
template <int D, int U>
__device__ __forceinline__ void vmwait_group(int g) {
    static_assert(D <= 8 && 2 * U * (D - 1) <= 63, "vmcnt holds 6 bits");
    if (g >= D - 1) {
        vmwait<2 * U * (D - 1)>();
        return;
    }
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
template <int U, int L>
__device__ __forceinline__ void ring_step(double (&t)[U], const double (&c)[U][2], const double (&pr)[64]) {
    constexpr int e = L & 1, n = (L & 31) >> 1;
#pragma unroll
    for (int u = 0; u < U; ++u) fmac_bc<n>(t[u], c[u][e], pr[L]);
}
template <int U, int L0, int... I>
__device__ __forceinline__ void ring_half(double (&t)[U], const double (&c)[U][2], const double (&pr)[64],
                                          std::integer_sequence<int, I...>) {
    (ring_step<U, L0 + I>(t, c, pr), ...);
}

// PUB: band publication as form 21's (pass_d_kernel)
template <bool NT, int U, int D, bool PUB = false>
__global__ __launch_bounds__(256) void pass_q_kernel(const double* __restrict__ T, double* __restrict__ Tout,
                                                     int64_t ld, int64_t rows, int64_t width,
                                                     const BlockDesc* __restrict__ bd,
                                                     const double* __restrict__ C, int64_t ldc,
                                                     const double* __restrict__ P,
                                                     const int32_t* __restrict__ nzc, int rb,
                                                     uint32_t* bcnt = nullptr) {
    constexpr int K = 64, SLOT = 128 * U;   // doubles per ring slot
    constexpr int kSt = (NT ? 2 : 0) | (PUB ? kAuxSc1 : 0);   // store policy
    static_assert(U % 2 == 0, "one DMA carries two rows");
    __shared__ int32_t cls[1024];
    extern __shared__ double ring[];   // [4 waves][D slots][SLOT]
    const int kb = bd->blk;
    const bool outplace = Tout != T;
    if (kb == 0 && !outplace) return;   // full and partial blocks alike (zeroed tails)
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool colok = j < width;
    const int jc = (int)(colok ? j : width - 1);
    double pr[K];   // all 64 rows: a partial block's P[l >= kb] is +0 (zeroed at block start)
#pragma unroll
    for (int l = 0; l < K; ++l) pr[l] = P[(int64_t)l * ld + jc];
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    classify_band(cls, bd, nzc, i0, nr, kb);
    __syncthreads();
    // the P loads complete here, before the ring starts (else hipcc waits for them, and
    // with them for everything, at the top of every group)
#pragma unroll
    for (int l = 0; l < K; ++l) asm volatile("" ::"v"(pr[l]));
    const int ng = (nr + U - 1) / U;
    // DMA sources: this lane's row of each DMA (row 2k + lane / 32 of a group, clamped to the
    // band) and its 16 B of the wave's 64 columns (clamped inside the row stride) / of the
    // row's 64 coefficients
    const int64_t wc = (int64_t)blockIdx.x * 256 + w * 64 + 2 * (lane & 31);
    const int64_t wcc = wc < ld - 1 ? wc : ld - 2;
    const double* tsrc = T + i0 * ld + wcc;
    const double* csrc = C + i0 * ldc + 2 * (lane & 31);
    double* wbase = ring + (size_t)w * D * SLOT;
    const uint32_t lbase = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)wbase;
    auto dma = [&](int g, int s) {
        const int gg = g < ng ? g : ng - 1;
#pragma unroll
        for (int k = 0; k < U / 2; ++k) {
            int r = gg * U + 2 * k + (lane >> 5);
            r = r < nr ? r : nr - 1;
            glds16(tsrc + (int64_t)r * ld, __builtin_amdgcn_readfirstlane(lbase + s * SLOT * 8 + k * 1024));
        }
#pragma unroll
        for (int k = 0; k < U / 2; ++k) {
            int r = gg * U + 2 * k + (lane >> 5);
            r = r < nr ? r : nr - 1;
            glds16(csrc + (int64_t)r * ldc,
                   __builtin_amdgcn_readfirstlane(lbase + s * SLOT * 8 + U * 512 + k * 1024));
        }
    };
    // band descriptor (the caller keeps rb * ld * 8 < 2^31): rows at soffset r * ld8; stores
    // of lanes past the width, and of rows with nothing to store, go out of range (dropped)
    const int ld8 = (int)(ld * 8);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Tout + i0 * ld), (short)0, (int)((int64_t)nr * ld * 8), 0x00020000);
    const int voff_st = colok ? jc * 8 : 0x7fffff00;
    auto store = [&](double v, int r, bool keep) {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), ro, keep ? voff_st : 0x7fffff00,
                                              (r < nr ? r : 0) * ld8, kSt);
    };
#pragma unroll
    for (int s = 0; s < D; ++s) dma(s, s);
    int s = 0;
    for (int g = 0; g < ng; ++g) {
        vmwait_group<D, U>(g);
        const double* sl = wbase + s * SLOT;
        const int r0 = g * U;
        bool dense = r0 + U <= nr;
#pragma unroll
        for (int u = 0; u < U; ++u) dense = dense && cls[r0 + u < nr ? r0 + u : 0] == kDense;
        if (dense) {   // (uniform)
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
            loadc(0);
            ring_half<U, 0>(t, c, pr, std::make_integer_sequence<int, 32>{});
            loadc(1);
            ring_half<U, 32>(t, c, pr, std::make_integer_sequence<int, 32>{});
#pragma unroll
            for (int u = 0; u < U; ++u) store(t[u], r0 + u, true);
        } else {
            // generic replay, row by row (form 21's); exactly U stores for the counted waits
            for (int u = 0; u < U; ++u) {
                const int r = r0 + u;
                const int cl = r < nr ? cls[r] : kUntouched;
                double t = sl[u * 64 + lane];
                if (cl == kUntouched) {
                    store(t, r, outplace && r < nr);
                    continue;
                }
                const double* cr = sl + U * 64 + u * 64;   // the row's coefficients (broadcast reads)
                t = replay_row(t, cl, pr, [&](int l) { return cr[l]; });
                store(t, r, true);
            }
        }
        dma(g + D, s);
        s = s + 1 == D ? 0 : s + 1;
    }
    if constexpr (PUB) {
        vmwait<0>();   // every wave: its sc1 stores are through (and the clamped tail DMAs landed)
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(&bcnt[blockIdx.y], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}


// Form 22: the K = 64 pass on the matrix cores.  v_mfma_f64_16x16x4f64 rounds exactly as
// four sequential fmas in k order (tools/mfma_probe.hip: 51.2 M random elements, denormal
// and signed-zero operands included), so T_tile := mfma(-C_frag, P_frag, T_tile) over the
// 16 k-blocks of a block is the eager sequence t = fma(-C[i][l], P[l][c], t), l = 0..63.
// Workgroup: 4 waves x NT 16-column tiles (64 NT columns) of a band; each wave keeps the
// P fragments of its tiles (16 x NT doubles per lane) for the band; the 4 waves share
// each 16-row group, whose coefficient rows are staged in LDS (rows padded to 66 doubles:
// conflict-free A-fragment reads) by LDS-DMA with per-lane source addresses, one group
// ahead, next to the next group's T tiles in registers.  Accumulator layout: lane l, reg i
// = row l/16 + 4 i, column l%16.  Every group runs through the MFMAs; only rows of class
// dense are stored, the rest (the block's pivot rows, sparse rows; copies of untouched
// rows out of place) go through the generic replay afterwards.  Partial blocks run the
// same code (tails zeroed at block start).
typedef double d4 __attribute__((ext_vector_type(4)));
// PUB (lookahead, round 5): band publication as form 21's — every output store write-through
// (sc1, beside nt) through a band buffer resource, every wave drained, then one agent-scope add
// to the band's count (pass_d_kernel).  The caller keeps rb * ld * 8 < 2^31.
template <bool NT_, int NT, bool PUB = false>
__global__ __launch_bounds__(256, 2) void pass_m_kernel(const double* __restrict__ T, double* __restrict__ Tout,
                                                     int64_t ld, int64_t rows, int64_t width,
                                                     const BlockDesc* __restrict__ bd,
                                                     const double* __restrict__ C, int64_t ldc,
                                                     const double* __restrict__ P,
                                                     const int32_t* __restrict__ nzc, int rb,
                                                     uint32_t* bcnt = nullptr) {
    constexpr int kSt = (NT_ ? 2 : 0) | (PUB ? kAuxSc1 : 0);   // store policy (PUB)
    constexpr int K = 64, KB = K / 4, W = 16 * NT, RS = K + 2;
    constexpr int NPC = (16 * RS + 127) / 128;   // 1 KiB LDS-DMA pieces per group
    // ONE __shared__ object (the coefficient stages, then the row classes): with a second one
    // beside the LDS-DMA target, hipcc waits vmcnt(0) before the class reads of the stores,
    // draining the next group's prefetch every group (cdna_hip_programming.md, glds traps)
    __shared__ double lds_all[2 * NPC * 128 + 512];
    double(*As)[NPC * 128] = reinterpret_cast<double(*)[NPC * 128]>(lds_all);
    int32_t* cls = reinterpret_cast<int32_t*>(lds_all + 2 * NPC * 128);
    const int kb = bd->blk;
    const bool outplace = Tout != T;
    if (kb == 0 && !outplace) return;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lr = lane & 15, lq = lane >> 4;
    const int64_t cw = (int64_t)blockIdx.x * (4 * W);   // the workgroup's first column
    const int64_t c0 = cw + w * W;
    double b[KB][NT];   // P fragments: rows 4 b + lq, column c0 + 16 t + lr
#pragma unroll
    for (int k4 = 0; k4 < KB; ++k4)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int64_t col = c0 + 16 * t + lr;
            b[k4][t] = P[(int64_t)(4 * k4 + lq) * ld + (col < width ? col : width - 1)];
        }
    const int64_t i0 = (int64_t)blockIdx.y * rb;
    const int64_t iend = (i0 + rb < rows) ? i0 + rb : rows;
    const int nr = (int)(iend - i0);
    classify_band(cls, bd, nzc, i0, nr, kb);
    const int ng = (nr + 15) / 16;
    // PUB: the band's output through one buffer resource (byte offsets column * 8 + row * ld8;
    // the caller keeps rb * ld * 8 < 2^31)
    const int ld8 = (int)(ld * 8);
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(Tout + i0 * ld), (short)0, (int)((int64_t)nr * ld * 8), 0x00020000);
    (void)ro;
    (void)ld8;
    auto stage = [&](int g, int buf) {
        const int gg = g < ng ? g : ng - 1;
        for (int pc = w; pc < NPC; pc += 4) {
            const int e0 = pc * 128 + 2 * lane;   // this lane's LDS doubles e0, e0 + 1
            int r = e0 / RS, c = e0 % RS;
            if (c >= K || r >= 16) {   // padding: any valid source
                r = 0;
                c = 0;
            }
            int64_t row = i0 + (int64_t)gg * 16 + r;
            row = row < iend ? row : iend - 1;
            __builtin_amdgcn_global_load_lds(C + row * ldc + c,
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
                acc[t][i] = NT_ ? __builtin_nontemporal_load(T + row * ld + cc) : T[row * ld + cc];
            }
        }
    };
    d4 ta[NT], tb[NT];
    stage(0, 0);
    loadt(ta, 0);
    constexpr int STG = (NPC + 3) / 4;   // staging instructions per wave per group
    for (int g = 0; g < ng; g += 2) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int gg = g + h;
            if (gg >= ng) break;
            d4(&acc)[NT] = h == 0 ? ta : tb;
            d4(&nxt)[NT] = h == 0 ? tb : ta;
            // cls is complete; buffer (gg + 1) & 1 is free (group gg - 1 done).  Raw barriers: a
            // __syncthreads() waits vmcnt(0), which would drain the prefetch issued below
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            stage(gg + 1, (gg + 1) & 1);
            loadt(nxt, gg + 1);
            // this group's staging and tile: all but the loads just issued
            constexpr int NEWV = NT * 4 + STG;
            __builtin_amdgcn_s_waitcnt(0x3F70 | (NEWV & 0xF) | ((NEWV >> 4) << 14));
            asm volatile("s_barrier" ::: "memory");   // every wave's pieces of this group landed
            const double* a = &As[gg & 1][lr * RS + lq];
#pragma unroll
            for (int k4 = 0; k4 < KB; ++k4) {
                const double av = -a[4 * k4];
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, b[k4][t], acc[t], 0, 0, 0);
            }
            const int rl0 = gg * 16;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int64_t col = c0 + 16 * t + lr;
                if (col < width)
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int rl = rl0 + lq + 4 * i;
                        if (rl < nr && cls[rl] == kDense) {
                            if constexpr (PUB) {   // (per-lane row: in the VGPR offset, not the SGPR one)
                                const double v = acc[t][i];
                                __builtin_amdgcn_raw_buffer_store_b64(dbits(v), ro,
                                                                      (int)col * 8 + (lq + 4 * i) * ld8, rl0 * ld8,
                                                                      kSt);
                            } else {
                                double* q = Tout + (i0 + rl) * ld + col;
                                if (NT_)
                                    __builtin_nontemporal_store(acc[t][i], q);
                                else
                                    *q = acc[t][i];
                            }
                        }
                    }
            }
        }
    }
    // everything else, row by row (as pass_s_body's generic replay): the 256 threads as
    // 256 / WC row slices x the workgroup's WC = 4 W columns
    constexpr int WC = 4 * W;
    const int64_t j = cw + (threadIdx.x % WC);
    const bool jok = j < width && threadIdx.x < (256 / WC) * WC;
    for (int r = threadIdx.x / WC; jok && r < nr; r += 256 / WC) {
        const int cl = cls[r];
        if (cl == kDense || (cl == kUntouched && !outplace)) continue;
        const double* row = T + (i0 + r) * ld;
        double t;
        if (cl == kUntouched) {
            t = row[j];
        } else {
            int l = 0;
            if (cl >= 0) {
                t = P[(int64_t)cl * ld + j];
                l = cl + 1;
            } else {
                t = row[j];
            }
            const double* cr = C + (i0 + r) * ldc;
            for (; l < kb; ++l) {
                const double f = cr[l];
                if (f != 0.0) t = __builtin_fma(-f, P[(int64_t)l * ld + j], t);
            }
        }
        if constexpr (PUB)   // (r differs between the lanes: VGPR offset)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, t), ro, (int)j * 8 + r * ld8, 0, kSt);
        else
            Tout[(i0 + r) * ld + j] = t;
    }
    if constexpr (PUB) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave: its sc1 stores are through
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(&bcnt[blockIdx.y], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void blk_reset_kernel(DevState* st) {
    if (threadIdx.x == 0) {
        st->blk = 0;
        st->bser = st->bser + 1;   // (condensed tableau: the next block's restarts are its own)
    }
}

// Condensed tableau: before a block's pass, each slot restarted in the block gets the unit
// vector of its new variable (1 in the step's pivot row, +0 elsewhere) in the pass's INPUT, in
// step order (a slot restarted twice keeps the later one): the pass then replays every step on it,
// the steps before the restart being no-ops (their P entries of the slot were zeroed by the
// commit).  One lane per local row; a column write, 8 B per row per restart.
__global__ __launch_bounds__(256) void reset_cols_kernel(double* __restrict__ T, int64_t ld, int64_t rows,
                                                         const int32_t* __restrict__ blkp,
                                                         const int32_t* __restrict__ pl,
                                                         const int32_t* __restrict__ qs) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows) return;
    const int kb = *blkp;
    double* r = T + i * ld;
    for (int l = 0; l < kb; ++l) r[qs[l]] = (pl[l] == (int32_t)i) ? 1.0 : 0.0;
}

// Lookahead: the block just selected becomes st->seal[slot] (read by its pass and
// replayed by the next block's selections); the next block starts empty.
// (bcnt: the slot's band counts restart at 0 for the pass about to be launched, whose
// output the next block's selections poll; the slot's previous pass has finished.)
__global__ __launch_bounds__(64) void seal_kernel(DevState* st, int slot, uint32_t* bcnt, int64_t nb) {
    const int kb = st->blk;
    for (int l = threadIdx.x; l < kMaxDefer; l += 64) {
        st->seal[slot].pl[l] = l < kb ? st->pl[l] : -1;
        st->seal[slot].qs[l] = st->qs[l];
    }
    if (bcnt)
        for (int64_t b = threadIdx.x; b < nb; b += 64) bcnt[b] = 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        st->seal[slot].blk = kb;
        st->seal[slot].ser = st->bser;
        st->blk = 0;
        st->bser = st->bser + 1;
    }
}

}  // namespace

// Rows per wave of the grouped ring.  In isolation (chainlab, cold inputs, 127 / 64 replayed steps)
// it replays 1.6-2x faster than the LEAN ring: 64 rows per wave on 256-lane workgroups (C3 rows on
// 64 CUs: 20.4 / 10.0 us vs 36.4 / 14.0), 32 on the rank geometries' 128-lane ones (c3r4 on 128
// CUs: 11.9 / 6.8 vs 22.6 / 11.5; profiles/r06q/-r06s/).  In the product the selection launch is
// bound by its other round trips, so the pivot rate barely moves (profiles/r06t/, alternating):
// c3r2 +1.5% (both pairs), C3 equal (pass-bound), c3r4 equal, c3r8 -1.5% (both pairs).  Auto: the
// grouped ring on 256-lane workgroups, the LEAN ring on 128-lane ones.
static int ratio_ring_rows(const Geometry& g) {
    return g.rthreads >= 256 ? 64 : 0;
}

int ratio_defer_blocks(const Geometry& g) {
    return (int)((g.rows + 1 + g.rthreads - 1) / g.rthreads);
}
// the fused single-rank pivot and the one-launch peer pivot keep 256-lane ratio workgroups
static int ratio_blocks_256(const Geometry& g) {
    return (int)((g.rows + 1 + kRatioDeferThreads - 1) / kRatioDeferThreads);
}

hipError_t launch_ratio_defer(const Geometry& g, const Defer& d, int32_t* basis,
                              const PricePart* pp, DevState* st, Cand* partials, int nblocks,
                              Cand* cand_out, int nranks, double tol_dj, double tol_piv,
                              int pricing, dlp_pivot* log, int64_t log_cap, hipStream_t s,
                              const Defer* prev, int prev_seal, const XPeers* xp, uint32_t xseq,
                              const BandPub* bp, bool xfuse, bool own_cus) {
    const int ntiles = (int)((g.width + kDeferTile - 1) / kDeferTile);
    const bool pub = bp && bp->cnt && bp->Tn && prev_seal >= 0;
    xfuse = xfuse && xp && nranks > 1;
    if (nblocks < ratio_defer_blocks(g)) return hipErrorInvalidValue;   // partials too small
    nblocks = ratio_defer_blocks(g);
    if (prev_seal >= 0 && (!prev || prev_seal > 1 || 2 * d.K > kMaxReplay)) return hipErrorInvalidValue;
    const double* Ccp = prev_seal >= 0 ? prev->Cc : nullptr;
    const double* Pp = prev_seal >= 0 ? prev->P : nullptr;
    const int steps = prev_seal >= 0 ? 2 * d.K : d.K;   // at most kp + j replayed steps
    if (g.rthreads != 64 && g.rthreads != 128 && g.rthreads != 256) return hipErrorInvalidValue;
#define DLP_RATIO_DEFER(KM)                                                                      \
    ratio_defer_kernel<KM><<<nblocks, g.rthreads, 0, s>>>(                               \
        g.T, g.ld, g.rows, g.rows_elig, g.ncols, g.row_first, basis, pp, ntiles, st, d.C, d.ldc, \
        d.Cc, d.ldcc, d.P, d.rhs, d.nzc, partials, cand_out, nranks, tol_dj, tol_piv, pricing,   \
        log, log_cap, Ccp, Pp, prev_seal, xp, xseq, xfuse ? 1 : 0, g.cd)
    if (steps <= 8)
        DLP_RATIO_DEFER(8);
    else if (steps <= 16)
        DLP_RATIO_DEFER(16);
    else if (steps <= 32)
        DLP_RATIO_DEFER(32);
    else if (steps <= 64)
        DLP_RATIO_DEFER(64);
    else   // lookahead at K = 64, beside the form-21 pass
    {
        static const int lch = std::getenv("DLP_LEAN_LCH") ? std::atoi(std::getenv("DLP_LEAN_LCH")) : 0;
        static const int mid_env = std::getenv("DLP_MID_CHAIN") ? std::atoi(std::getenv("DLP_MID_CHAIN")) : -1;
        if (mid_env >= 0 ? mid_env == 1 : d.form == 22) {   // beside the MFMA pass: registers, no ring
            ratio_mid_kernel<128, 16><<<nblocks, g.rthreads, 0, s>>>(
                g.T, g.ld, g.rows, g.rows_elig, g.ncols, g.row_first, basis, pp, ntiles, st, d.C, d.ldc, d.Cc, d.ldcc,
                d.P, d.rhs, d.nzc, partials, cand_out, nranks, tol_dj, tol_piv, pricing, log, log_cap, Ccp, Pp,
                prev_seal, xp, xseq, pub ? bp->cnt + prev_seal * bp->stride : nullptr, pub ? bp->rb : 1,
                pub ? bp->ntiles : 0, pub ? bp->Tn : nullptr, xfuse ? 1 : 0, g.cd);
            return hipGetLastError();
        }
        // the chain on CUs of its own: the grouped ring, ROWS rows per wave (DLP_RATIO_ROWS = 64 / 32 / 16
        // overrides the policy, 0 keeps the LEAN ring)
        static const int rows_env = std::getenv("DLP_RATIO_ROWS") ? std::atoi(std::getenv("DLP_RATIO_ROWS")) : -1;
        const int rrows = rows_env >= 0 ? rows_env : (own_cus ? ratio_ring_rows(g) : 0);
        if (rrows == 64 || rrows == 32 || rrows == 16) {
            const int lanes = g.rthreads * 64 / rrows;
            if (lanes > 1024) return hipErrorInvalidValue;
#define DLP_RATIO_RING(R_, RP_, RG_)                                                                         \
    ratio_ring_kernel<R_, RP_, RG_><<<nblocks, lanes, (size_t)(lanes / 64) * RP_ * 1024, s>>>(                 \
        g.T, g.ld, g.rows, g.rows_elig, g.ncols, g.row_first, basis, pp, ntiles, st, d.C, d.ldc, d.Cc, d.ldcc, \
        d.P, d.rhs, d.nzc, partials, cand_out, nranks, tol_dj, tol_piv, pricing, log, log_cap, Ccp, Pp, prev_seal, \
        xp, xseq, pub ? bp->cnt + prev_seal * bp->stride : nullptr, pub ? bp->rb : 1, pub ? bp->ntiles : 0,   \
        pub ? bp->Tn : nullptr, xfuse ? 1 : 0, g.cd)
            // (DLP_RATIO_RP=12: 12 DMAs in flight, 48 KB of ring per 256-lane workgroup, so three share a
            // CU and C3's 129 workgroups are resident at once on 64 CUs; tuning)
            static const int rp_env = std::getenv("DLP_RATIO_RP") ? std::atoi(std::getenv("DLP_RATIO_RP")) : 16;
            if (rrows == 64 && rp_env == 12)
                DLP_RATIO_RING(64, 12, 4);
            else if (rrows == 64)
                DLP_RATIO_RING(64, 16, 4);
            else if (rrows == 32)
                DLP_RATIO_RING(32, 16, 4);
            else
                DLP_RATIO_RING(16, 16, 2);
#undef DLP_RATIO_RING
            return hipGetLastError();
        }
        static const int ring_env = std::getenv("DLP_CHAIN_RING") ? std::atoi(std::getenv("DLP_CHAIN_RING")) : 0;
#define DLP_RATIO_LEAN(L, DYN, ...)                                                                        \
    ratio_lean_kernel<128, L, ##__VA_ARGS__><<<nblocks, g.rthreads, DYN, s>>>(                         \
        g.T, g.ld, g.rows, g.rows_elig, g.ncols, g.row_first, basis, pp, ntiles, st, d.C, d.ldc, d.Cc, d.ldcc, \
        d.P, d.rhs, d.nzc, partials, cand_out, nranks, tol_dj, tol_piv, pricing, log, log_cap, Ccp, Pp, prev_seal, \
        xp, xseq, pub ? bp->cnt + prev_seal * bp->stride : nullptr, pub ? bp->rb : 1, pub ? bp->ntiles : 0,   \
        pub ? bp->Tn : nullptr, xfuse ? 1 : 0, g.cd)
        // the LDS ring (0); 4 or 8 coefficient loads per round trip for tuning only (DLP_LEAN_LCH)
        if (lch == 8 && !g.cd.on)
            DLP_RATIO_LEAN(8, 0);
        else if (lch == 4)
            DLP_RATIO_LEAN(4, 0);
        else if (ring_env == 16)   // (tuning: DLP_CHAIN_RING=16, 16 ring DMAs in flight per wave)
            DLP_RATIO_LEAN(0, ratio_ring_bytes(16) / (kRatioDeferThreads / g.rthreads), 16);
        else
            DLP_RATIO_LEAN(0, ratio_ring_bytes(kRatioRingPairs) / (kRatioDeferThreads / g.rthreads));
#undef DLP_RATIO_LEAN
    }
#undef DLP_RATIO_DEFER
    return hipGetLastError();
}

hipError_t launch_pivot_defer(const Geometry& g, const Defer& d, int32_t* basis, PricePart* pp,
                              DevState* st, Cand* partials, int nblocks, double tol_dj,
                              double tol_piv, int pricing, dlp_pivot* log, int64_t log_cap,
                              hipStream_t s) {
    const int ntiles = (int)((g.width + kDeferTile - 1) / kDeferTile);
    if (nblocks < ratio_blocks_256(g)) return hipErrorInvalidValue;   // partials too small
    const int nrat = ratio_blocks_256(g);
    const int nprow = (int)((g.ld + kDeferTile - 1) / kDeferTile);
    // every block resident at once (the pivot-row blocks wait on the ratio blocks): the
    // caller keeps the grid within 2 blocks per CU (fused_pivot_fits); K <= 32
    if (d.K > 32 || g.cd.on) return hipErrorInvalidValue;   // (no condensed-tableau instance)
#define DLP_PIVOT_DEFER(KM)                                                                       \
    pivot_defer_kernel<KM><<<nrat + nprow, 256, 0, s>>>(                                          \
        g.T, g.ld, g.rows, g.rows_elig, g.ncols, g.nprice, g.row_first, basis, pp, ntiles, st,    \
        d.C, d.ldc, d.Cc, d.ldcc, d.P, d.rhs, d.nzc, partials, nrat, tol_dj, tol_piv, pricing,    \
        log, log_cap)
    if (d.K <= 8)
        DLP_PIVOT_DEFER(8);
    else if (d.K <= 16)
        DLP_PIVOT_DEFER(16);
    else
        DLP_PIVOT_DEFER(32);
#undef DLP_PIVOT_DEFER
    return hipGetLastError();
}

int fused_pivot_blocks(const Geometry& g) {
    return ratio_blocks_256(g) + (int)((g.ld + kDeferTile - 1) / kDeferTile);
}

// How many workgroups of the fused pivot kernel (the instance launch_pivot_defer picks for K)
// the device holds at once, from the compiled kernel's real occupancy (0 when unknown): its
// pivot-row blocks spin on the ratio blocks' selection, so the whole grid must be resident.
int fused_pivot_capacity(int K, int cus) {
    int per = 0;
    const hipError_t e =
        K <= 8    ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pivot_defer_kernel<8>, 256, 0)
        : K <= 16 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pivot_defer_kernel<16>, 256, 0)
                  : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pivot_defer_kernel<32>, 256, 0);
    return e == hipSuccess ? per * cus : 0;
}

hipError_t launch_prow_defer(const Geometry& g, const Defer& d, const DevState* st,
                             int64_t* prow_bits, PricePart* pp, double tol_dj, dlp_pivot* log,
                             int64_t log_cap, int nranks, hipStream_t s, const Defer* prev,
                             int prev_seal, const XPeers* xp, uint32_t xseq, const BandPub* bp,
                             bool xfuse, bool own_cus) {
    const int blocks = (int)((g.ld + kDeferTile - 1) / kDeferTile);
    const int xc = (xfuse && xp && nranks > 1) ? 1 : 0;
    if (prev_seal >= 0 && (!prev || prev_seal > 1 || 2 * d.K > kMaxReplay)) return hipErrorInvalidValue;
    const bool pub = bp && bp->cnt && bp->Tn && prev_seal >= 0;
    static const int fat_env = std::getenv("DLP_FAT_PROW") ? std::atoi(std::getenv("DLP_FAT_PROW")) : -1;
    // the chain on CUs of its own: the grouped ring (DLP_PROW_GROUP = 4) or the register kernel
    static const int pg_env = std::getenv("DLP_PROW_GROUP") ? std::atoi(std::getenv("DLP_PROW_GROUP")) : 0;
    if (prev_seal >= 0 && d.K > 32 && own_cus && fat_env < 0 && pg_env == 4) {
        prow_ring_kernel<16, 4><<<blocks, 256, prow_ring_bytes(16), s>>>(
            g.T, g.ld, g.rows, g.ncols, g.nprice, st, d.C, d.ldc, d.P, prow_bits, pp, tol_dj, log, log_cap,
            nranks == 1 ? 1 : 0, prev->C, prev->P, prev_seal, nranks == 1 ? nullptr : xp, xseq,
            pub ? bp->cnt + prev_seal * bp->stride : nullptr, pub ? bp->rb : 1, pub ? bp->ntiles : 0,
            pub ? bp->Tn : nullptr, xc, g.cd);
        return hipGetLastError();
    }
    const bool fat = fat_env >= 0 ? fat_env == 1 : own_cus;
    static const int mid_env = std::getenv("DLP_MID_CHAIN") ? std::atoi(std::getenv("DLP_MID_CHAIN")) : -1;
    const bool mid = !fat && (mid_env >= 0 ? mid_env == 1 : d.form == 22);
    if (prev_seal >= 0 && d.K > 32 && mid) {
        // beside the MFMA pass (form 22 leaves 104 VGPRs per SIMD): the register replay, 2 x 8 rows
        prow_mid_kernel<<<blocks, 256, 0, s>>>(g.T, g.ld, g.rows, g.ncols, g.nprice, st, d.C, d.ldc, d.P, prow_bits,
                                              pp, tol_dj, log, log_cap, nranks == 1 ? 1 : 0, prev->C, prev->P,
                                              prev_seal, nranks == 1 ? nullptr : xp, xseq,
                                              pub ? bp->cnt + prev_seal * bp->stride : nullptr, pub ? bp->rb : 1,
                                              pub ? bp->ntiles : 0, pub ? bp->Tn : nullptr, xc, g.cd);
    } else if (prev_seal >= 0 && d.K > 32 && fat) {
        // lookahead with the chain on CUs of its own (no pass waves beside it): the register
        // kernel, 2 x 16 pivot rows in flight, with band publication
        prow_defer_kernel<<<blocks, 256, 0, s>>>(g.T, g.ld, g.rows, g.ncols, g.nprice, st, d.C, d.ldc, d.P, prow_bits,
                                                 pp, tol_dj, log, log_cap, nranks == 1 ? 1 : 0, prev->C, prev->P,
                                                 prev_seal, nranks == 1 ? nullptr : xp, xseq,
                                                 pub ? bp->cnt + prev_seal * bp->stride : nullptr, pub ? bp->rb : 1,
                                                 pub ? bp->ntiles : 0, pub ? bp->Tn : nullptr, xc, g.cd);
    } else if (prev_seal >= 0 && d.K > 32) {   // lookahead at K = 64: beside the form-21 pass
#define DLP_PROW_LEAN(RS)                                                                                  \
    prow_lean_kernel<RS><<<blocks, 256, prow_ring_bytes(RS), s>>>(                                          \
        g.T, g.ld, g.rows, g.ncols, g.nprice, st, d.C, d.ldc, d.P, prow_bits, pp, tol_dj, log, log_cap,     \
        nranks == 1 ? 1 : 0, prev->C, prev->P, prev_seal, nranks == 1 ? nullptr : xp, xseq,                \
        pub ? bp->cnt + prev_seal * bp->stride : nullptr, pub ? bp->rb : 1, pub ? bp->ntiles : 0,           \
        pub ? bp->Tn : nullptr, xc, g.cd)
        static const int ring_env = std::getenv("DLP_CHAIN_RING") ? std::atoi(std::getenv("DLP_CHAIN_RING")) : 0;
        if (ring_env == 16)
            DLP_PROW_LEAN(16);
        else
            DLP_PROW_LEAN(kProwRingSteps);
#undef DLP_PROW_LEAN
    } else
        prow_defer_kernel<<<blocks, 256, 0, s>>>(g.T, g.ld, g.rows, g.ncols, g.nprice, st, d.C, d.ldc,
                                                 d.P, prow_bits, pp, tol_dj, log, log_cap,
                                                 nranks == 1 ? 1 : 0, prev_seal >= 0 ? prev->C : nullptr,
                                                 prev_seal >= 0 ? prev->P : nullptr, prev_seal,
                                                 nranks == 1 ? nullptr : xp, xseq, nullptr, 1, 0, nullptr, xc, g.cd);
    return hipGetLastError();
}

hipError_t launch_pivot_x(const Geometry& g, const Defer& d, int32_t* basis, PricePart* pp, DevState* st,
                          double tol_dj, double tol_piv, int pricing, dlp_pivot* log, int64_t log_cap,
                          hipStream_t s, const Defer* prev, int prev_seal, const XPeers* xp, uint32_t seq,
                          const BandPub* bp, bool own_cus) {
    // 256-lane ratio blocks (the ring instance: 128 or 256 rows each, on the chain's own CUs); the
    // selection record carries the condensed tableau's entering slot
    const bool ring = own_cus && d.K == 64 && (g.rthreads == 128 || g.rthreads == kRatioDeferThreads);
    if (!xp || (!ring && g.rthreads != kRatioDeferThreads)) return hipErrorInvalidValue;
    if (prev_seal >= 0 && (!prev || prev_seal > 1 || 2 * d.K > kMaxReplay)) return hipErrorInvalidValue;
    const int ntiles = (int)((g.width + kDeferTile - 1) / kDeferTile);
    const int nrat = ratio_defer_blocks(g);
    const int nprow = (int)((g.ld + kDeferTile - 1) / kDeferTile);
    const bool pub = bp && bp->cnt && bp->Tn && prev_seal >= 0;
    const double* Ccp = prev_seal >= 0 ? prev->Cc : nullptr;
    const double* Pp = prev_seal >= 0 ? prev->P : nullptr;
    const double* Cp = prev_seal >= 0 ? prev->C : nullptr;
    const int steps = prev_seal >= 0 ? 2 * d.K : d.K;
#define DLP_PX_ARGS                                                                                          \
    g.T, g.ld, g.rows, g.rows_elig, g.ncols, g.nprice, g.row_first, basis, pp, ntiles, st, d.C, d.ldc, d.Cc, \
        d.ldcc, d.P, d.rhs, d.nzc, nrat, tol_dj, tol_piv, pricing, log, log_cap, Ccp, Pp, Cp, prev_seal, xp, \
        seq, pub ? bp->cnt + prev_seal * bp->stride : nullptr, pub ? bp->rb : 1, pub ? bp->ntiles : 0,     \
        pub ? bp->Tn : nullptr, 2, g.cd
    if (!ring && steps > 64 && g.cd.on) return hipErrorInvalidValue;   // (the LEAN instance has no condensed build)
    if (ring) {
        if (g.rthreads == 128)
            pivot_x_ring_kernel<32><<<nrat + nprow, 256, (size_t)4 * 16 * 1024, s>>>(DLP_PX_ARGS);
        else
            pivot_x_ring_kernel<64><<<nrat + nprow, 256, (size_t)4 * 16 * 1024, s>>>(DLP_PX_ARGS);
    } else if (steps > 64)   // lookahead at K = 64, beside the form-21 pass
        pivot_x_lean_kernel<<<nrat + nprow, 256, std::max(ratio_ring_bytes(kRatioRingPairs),
                                                          prow_ring_bytes(kProwRingSteps)), s>>>(DLP_PX_ARGS);
    else if (steps <= 16)
        pivot_x_kernel<16><<<nrat + nprow, 256, 0, s>>>(DLP_PX_ARGS);
    else if (steps <= 32)
        pivot_x_kernel<32><<<nrat + nprow, 256, 0, s>>>(DLP_PX_ARGS);
    else
        pivot_x_kernel<64><<<nrat + nprow, 256, 0, s>>>(DLP_PX_ARGS);
#undef DLP_PX_ARGS
    return hipGetLastError();
}

hipError_t launch_commit_defer(const Geometry& g, const Defer& d, DevState* st,
                               const int64_t* prow_bits, PricePart* pp, double tol_dj,
                               dlp_pivot* log, int64_t log_cap, hipStream_t s, const XPeers* xp,
                               uint32_t xseq) {
    const int blocks = (int)((g.ld + kDeferTile - 1) / kDeferTile);
    commit_defer_kernel<<<blocks, 256, 0, s>>>(g.T, g.ld, g.rows, g.ncols, g.nprice, st, d.C,
                                               d.ldc, d.P, prow_bits, pp, tol_dj, log, log_cap, xp,
                                               xseq, g.cd);
    return hipGetLastError();
}

template <bool NT, int K, int V, int U, int D>
static void launch_pass_r(const Geometry& g, const Defer& d, DevState* st, int rb, size_t dyn,
                          int order, hipStream_t s) {
    const int ntiles = (int)((g.width + 256 * V - 1) / (256 * V));
    const int nbands = (int)((g.rows + rb - 1) / rb);
    const int64_t total = (int64_t)ntiles * nbands;
    const int64_t t8 = (ntiles + 7) / 8;
    const dim3 grid((unsigned)(order == 1 ? 8 * ((total + 7) / 8) : order == 2 ? 8 * t8 * nbands : total));
    pass_r_kernel<NT, K, V, U, D, false><<<grid, 256, dyn, s>>>(
        g.T, g.ld, g.rows, g.width, st, d.C, d.ldc, d.P, d.nzc, rb, ntiles, nbands, order);
    pass_r_kernel<NT, K, V, U, D, true><<<grid, 256, dyn, s>>>(
        g.T, g.ld, g.rows, g.width, st, d.C, d.ldc, d.P, d.nzc, rb, ntiles, nbands, order);
}

// DLP_PASS_LDS=<bytes> (tuning only): the dynamic LDS of the forms-21/23 pass workgroups, which caps
// how many share a CU while leaving the rest of the 160 KiB to the chain kernels beside them
static size_t pass_lds_env() {
    static const long v = std::getenv("DLP_PASS_LDS") ? std::atol(std::getenv("DLP_PASS_LDS")) : 0;
    return v > 0 && v <= 150 * 1024 ? (size_t)v : 0;
}

template <bool NT, int K>
static hipError_t pass(const Geometry& g, const Defer& d, DevState* st, int rb, int occ,
                       hipStream_t s, double* Tout, int seal, uint32_t* bcnt) {
    // lookahead: out of place, the sealed block; pass_s forms only (lookahead_form)
    if (seal >= 0 && !lookahead_form(d.form)) return hipErrorInvalidValue;
    const BlockDesc* bd = seal >= 0 ? &st->seal[seal] : (const BlockDesc*)&st->blk;
    double* To = Tout ? Tout : g.T;
    if (d.form >= 6 && d.form <= 19 && d.form != 14 && d.form != 15 &&
        (int64_t)rb * g.ld * 8 < ((int64_t)1 << 31)) {
        // streamed forms (K >= 16, a band within one 2 GiB buffer descriptor; else form 3)
        if constexpr (K >= 16) {
            if ((d.form == 6 || d.form == 7 || d.form == 10 || d.form == 11 || d.form == 16 ||
                 d.form == 17) && K > 32)
                return hipErrorInvalidValue;
            size_t dyn = 0;
            if (occ > 0) {   // static LDS: cls[1024], dgl[512], s_wtot[4]
                const size_t stat = 1024 * sizeof(int32_t) + 512 * sizeof(int16_t) + 16;
                dyn = (size_t)160 * 1024 / occ - stat;
            }
            if (g.rows > 0) {
                // forms 6-9: XCD work order by band groups; 10-13: the same with the
                // tile-fastest order; 16-19: XCD work order by tile ranges
                const int order = d.form <= 9 ? 1 : d.form <= 13 ? 0 : 2;
                const int f = d.form <= 9 ? d.form : d.form <= 13 ? d.form - 4 : d.form - 10;
                if (f == 6) {
                    if constexpr (K <= 32) launch_pass_r<NT, K, 2, 2, 4>(g, d, st, rb, dyn, order, s);
                } else if (f == 7) {
                    if constexpr (K <= 32) launch_pass_r<NT, K, 2, 2, 2>(g, d, st, rb, dyn, order, s);
                } else if (f == 8) {
                    launch_pass_r<NT, K, 1, 4, 4>(g, d, st, rb, dyn, order, s);
                } else {
                    launch_pass_r<NT, K, 1, 4, 2>(g, d, st, rb, dyn, order, s);
                }
            }
            blk_reset_kernel<<<1, 64, 0, s>>>(st);
            return hipGetLastError();
        }
    }
    if (d.form == 22 && K == 64 && d.K == 64 && d.ldc == 64 && rb <= 1024) {
        // MFMA pass (K = 64 blocks; 128-column workgroups)
        if constexpr (K == 64) {
            size_t dyn = 0;
            if (occ > 0) {
                const size_t stat = 1024 * sizeof(int32_t) + 2 * 9 * 128 * sizeof(double);
                dyn = (size_t)160 * 1024 / occ - stat;
            }
            const dim3 grid((unsigned)((g.width + 127) / 128), (unsigned)((g.rows + rb - 1) / rb));
            if (g.rows > 0) {
                if (bcnt && (int64_t)rb * g.ld * 8 < ((int64_t)1 << 31))
                    pass_m_kernel<NT, 2, true><<<grid, 256, dyn, s>>>(g.T, To, g.ld, g.rows, g.width, bd, d.C,
                                                                      d.ldc, d.P, d.nzc, rb, bcnt);
                else
                    pass_m_kernel<NT, 2><<<grid, 256, dyn, s>>>(g.T, To, g.ld, g.rows, g.width, bd, d.C, d.ldc,
                                                                 d.P, d.nzc, rb);
            }
            if (seal < 0) blk_reset_kernel<<<1, 64, 0, s>>>(st);
            return hipGetLastError();
        }
    }
    // (d.K == 64 exactly: the kernel addresses C with 64 steps per row, ldc == 64)
    if (d.form == 21 && K == 64 && d.K == 64 && d.ldc == 64 && (int64_t)rb * g.ld * 8 < ((int64_t)1 << 31) &&
        (int64_t)rb * d.ldc * 8 < ((int64_t)1 << 31)) {
        // DPP-coefficient pass (K = 64 blocks; 1 double per lane: 256-column tiles)
        if constexpr (K == 64) {
            size_t dyn = pass_lds_env();
            if (occ > 0) dyn = (size_t)160 * 1024 / occ - 1024 * sizeof(int32_t);
            const dim3 grid((unsigned)((g.width + 255) / 256), (unsigned)((g.rows + rb - 1) / rb));
            if (g.rows > 0) {
                if (bcnt)
                    pass_d_kernel<NT, true><<<grid, 256, dyn, s>>>(g.T, To, g.ld, g.rows, g.width, bd, d.C, d.ldc,
                                                                   d.P, d.nzc, rb, bcnt);
                else
                    pass_d_kernel<NT><<<grid, 256, dyn, s>>>(g.T, To, g.ld, g.rows, g.width, bd, d.C, d.ldc, d.P,
                                                             d.nzc, rb);
            }
            if (seal < 0) blk_reset_kernel<<<1, 64, 0, s>>>(st);
            return hipGetLastError();
        }
    }
    if (d.form == 23 && K == 64 && d.K == 64 && d.ldc == 64 && (int64_t)rb * g.ld * 8 < ((int64_t)1 << 31) &&
        rb <= 1024) {
        // LDS-ring DPP pass (K = 64 blocks; 256-column tiles): 2 rows per group, 4 groups in
        // flight per wave: 32 KiB of ring + 4 KiB of row classes per workgroup, so three pass
        // workgroups leave the lookahead chain's LDS free on a CU
        if constexpr (K == 64) {
            // ring depth D: 4 groups in flight (DLP_Q_DEPTH = 2 or 3: tuning only)
            static const int qd = std::getenv("DLP_Q_DEPTH") ? std::atoi(std::getenv("DLP_Q_DEPTH")) : 4;
            // rows per group: 4 (twice the independent fma chains per wave, 2 or 3 groups in flight)
            // from 16,384 rows, else 2 (alternating pairs, profiles/r06w/: C3 pass 4.455-4.458 vs
            // 4.519-4.523 ms, 13,951-13,956 vs 13,753-13,755 pivots/s; c3r2 equal; c3r4's pass 2%
            // slower with U = 4); DLP_Q_U = 2 / 4 overrides
            static const int qu_env = std::getenv("DLP_Q_U") ? std::atoi(std::getenv("DLP_Q_U")) : 0;
            const int qu = qu_env == 2 || qu_env == 4 ? qu_env : (g.rows >= 16384 ? 4 : 2);
            constexpr int U = 2;
            const int D = qd == 2 || qd == 3 || qd == 6 || qd == 8 ? qd : 4;
            if (qu == 4) {
                const int D4 = qd == 3 ? 3 : 2;
                size_t dyn4 = std::max((size_t)4 * D4 * 128 * 4 * sizeof(double), pass_lds_env());
                if (occ > 0) dyn4 = std::max(dyn4, (size_t)160 * 1024 / occ - 1024 * sizeof(int32_t));
                const dim3 grid4((unsigned)((g.width + 255) / 256), (unsigned)((g.rows + rb - 1) / rb));
                if (g.rows > 0) {
                    if (D4 == 3) {
                        if (bcnt)
                            pass_q_kernel<NT, 4, 3, true><<<grid4, 256, dyn4, s>>>(g.T, To, g.ld, g.rows, g.width, bd,
                                                                                d.C, d.ldc, d.P, d.nzc, rb, bcnt);
                        else
                            pass_q_kernel<NT, 4, 3><<<grid4, 256, dyn4, s>>>(g.T, To, g.ld, g.rows, g.width, bd, d.C,
                                                                          d.ldc, d.P, d.nzc, rb);
                    } else {
                        if (bcnt)
                            pass_q_kernel<NT, 4, 2, true><<<grid4, 256, dyn4, s>>>(g.T, To, g.ld, g.rows, g.width, bd,
                                                                                d.C, d.ldc, d.P, d.nzc, rb, bcnt);
                        else
                            pass_q_kernel<NT, 4, 2><<<grid4, 256, dyn4, s>>>(g.T, To, g.ld, g.rows, g.width, bd, d.C,
                                                                          d.ldc, d.P, d.nzc, rb);
                    }
                }
                if (seal < 0) blk_reset_kernel<<<1, 64, 0, s>>>(st);
                return hipGetLastError();
            }
            size_t dyn = std::max((size_t)4 * D * 128 * U * sizeof(double), pass_lds_env());
            if (occ > 0) dyn = std::max(dyn, (size_t)160 * 1024 / occ - 1024 * sizeof(int32_t));
            const dim3 grid((unsigned)((g.width + 255) / 256), (unsigned)((g.rows + rb - 1) / rb));
#define DLP_PASS_Q(DD)                                                                                     \
    do {                                                                                                   \
        if (bcnt)                                                                                          \
            pass_q_kernel<NT, U, DD, true><<<grid, 256, dyn, s>>>(g.T, To, g.ld, g.rows, g.width, bd, d.C, \
                                                                  d.ldc, d.P, d.nzc, rb, bcnt);           \
        else                                                                                               \
            pass_q_kernel<NT, U, DD><<<grid, 256, dyn, s>>>(g.T, To, g.ld, g.rows, g.width, bd, d.C, d.ldc, \
                                                           d.P, d.nzc, rb);                                \
    } while (0)
            if (g.rows > 0) {
                if (D == 2)
                    DLP_PASS_Q(2);
                else if (D == 3)
                    DLP_PASS_Q(3);
                else if (D == 6)
                    DLP_PASS_Q(6);
                else if (D == 8)
                    DLP_PASS_Q(8);
                else
                    DLP_PASS_Q(4);
            }
#undef DLP_PASS_Q
            if (seal < 0) blk_reset_kernel<<<1, 64, 0, s>>>(st);
            return hipGetLastError();
        }
    }
    // streamed forms need K >= 16 (an even number of coefficient chunks): form 3 below
    const int form = (d.form >= 6 && d.form != 14 && d.form != 15 && d.form != 20) ? 3 : d.form;
    const int cols = (form == 0 || form == 4 || form >= 14) ? kDeferTile : 256;
    const int ntiles = (int)((g.width + cols - 1) / cols);
    const int64_t bands = (g.rows + rb - 1) / rb;
    size_t dyn = form >= 3 ? 0 : (size_t)K * rb * sizeof(double) + (size_t)rb * sizeof(int32_t);
    if (dyn > 160 * 1024) return hipErrorInvalidValue;
    if (occ > 0) {   // reserve LDS so that at most `occ` workgroups fit on a CU (160 KiB)
        // the kernel's static LDS counts against the same 160 KiB: cls[1024] (forms 3-5),
        // s_pl[K] (forms 0-2)
        const size_t stat = form >= 14 ? 1024 * sizeof(int32_t) + 512 * sizeof(int16_t) + 16
                            : form >= 3 ? 1024 * sizeof(int32_t) : K * sizeof(int32_t);
        const size_t cap = (size_t)160 * 1024 / occ - stat;
        if (dyn < cap) dyn = cap;
    }
    const dim3 grid(ntiles, (unsigned)bands);
    // the session's K is this template's: partial blocks run the full-block instance (their
    // unused steps were zeroed at block start), one launch per pass
    const int tails = d.K == K ? 1 : 0;
    if (g.rows > 0) {
        if (form == 0) {
            if constexpr (K <= 32)   // 2 doubles per lane: P[0..K) in 4K VGPRs
                pass_kernel<NT, K><<<grid, 256, dyn, s>>>(g.T, g.ld, g.rows, g.width, st, d.C,
                                                          d.ldc, d.P, rb);
            else
                return hipErrorInvalidValue;
        } else if (form == 3) {
            pass_s_kernel<NT, K, 1, 4, false><<<grid, 256, dyn, s>>>(g.T, To, g.ld, g.rows, g.width, bd,
                                                                     d.C, d.ldc, d.P, d.nzc, rb, tails);
            if (!tails)
                pass_s_kernel<NT, K, 1, 4, true><<<grid, 256, dyn, s>>>(g.T, To, g.ld, g.rows, g.width, bd,
                                                                        d.C, d.ldc, d.P, d.nzc, rb, 0);
        } else if (form == 20) {
            if constexpr (K <= 32) {
                pass_s_kernel<NT, K, 2, 2, false, true><<<grid, 256, dyn, s>>>(
                    g.T, To, g.ld, g.rows, g.width, bd, d.C, d.ldc, d.P, d.nzc, rb, tails);
                if (!tails)
                    pass_s_kernel<NT, K, 2, 2, true><<<grid, 256, dyn, s>>>(
                        g.T, To, g.ld, g.rows, g.width, bd, d.C, d.ldc, d.P, d.nzc, rb, 0);
            } else
                return hipErrorInvalidValue;
        } else if (form == 4 || form == 14 || form == 15) {
            if constexpr (K <= 32) {
                // form 14 keeps its streamed partial-block kernel, form 15 (the 3-waves build,
                // which spills) its partial-block instance: its full-block build ran a partial
                // C3-geometry block with a wrong tableau (tests/test_gpu_defer.py)
                const int tl = (form == 14 || form == 15) ? 0 : tails;
                if (form == 15)
                    pass_s3_kernel<NT, K, 2, 2, false><<<grid, 256, dyn, s>>>(
                        g.T, To, g.ld, g.rows, g.width, bd, d.C, d.ldc, d.P, d.nzc, rb, tl);
                else
                    pass_s_kernel<NT, K, 2, 2, false><<<grid, 256, dyn, s>>>(
                        g.T, To, g.ld, g.rows, g.width, bd, d.C, d.ldc, d.P, d.nzc, rb, tl);
                if (form >= 14 && K >= 16 && (int64_t)rb * g.ld * 8 < ((int64_t)1 << 31)) {
                    // partial block through the streamed kernel's partial instance
                    const int nb = (int)bands;
                    if constexpr (K >= 16)
                        pass_r_kernel<NT, K, 2, 2, 4, true><<<dim3((unsigned)(ntiles * bands)), 256, dyn, s>>>(
                            g.T, g.ld, g.rows, g.width, st, d.C, d.ldc, d.P, d.nzc, rb, ntiles, nb, 0);
                } else if (!tl) {
                    pass_s_kernel<NT, K, 2, 2, true><<<grid, 256, dyn, s>>>(
                        g.T, To, g.ld, g.rows, g.width, bd, d.C, d.ldc, d.P, d.nzc, rb, 0);
                }
            } else
                return hipErrorInvalidValue;
        } else if (form == 5) {
            pass_s_kernel<NT, K, 1, 8, false><<<grid, 256, dyn, s>>>(g.T, To, g.ld, g.rows, g.width, bd,
                                                                     d.C, d.ldc, d.P, d.nzc, rb, tails);
            if (!tails)
                pass_s_kernel<NT, K, 1, 8, true><<<grid, 256, dyn, s>>>(g.T, To, g.ld, g.rows, g.width, bd,
                                                                        d.C, d.ldc, d.P, d.nzc, rb, 0);
        }
        else if (form == 1)
            pass1_kernel<NT, K, 2><<<grid, 256, dyn, s>>>(g.T, g.ld, g.rows, g.width, st, d.C,
                                                          d.ldc, d.P, rb);
        else
            pass1_kernel<NT, K, 4><<<grid, 256, dyn, s>>>(g.T, g.ld, g.rows, g.width, st, d.C,
                                                          d.ldc, d.P, rb);
    }
    if (seal < 0) blk_reset_kernel<<<1, 64, 0, s>>>(st);
    return hipGetLastError();
}

template <bool NT>
static hipError_t pass_k(const Geometry& g, const Defer& d, DevState* st, int rb, int occ,
                         hipStream_t s, double* Tout, int seal, uint32_t* bcnt) {
    if (d.K <= 4) return pass<NT, 4>(g, d, st, rb, occ, s, Tout, seal, nullptr);
    if (d.K <= 8) return pass<NT, 8>(g, d, st, rb, occ, s, Tout, seal, nullptr);
    if (d.K <= 16) return pass<NT, 16>(g, d, st, rb, occ, s, Tout, seal, nullptr);
    if (d.K <= 32) return pass<NT, 32>(g, d, st, rb, occ, s, Tout, seal, nullptr);
    return pass<NT, 64>(g, d, st, rb, occ, s, Tout, seal, bcnt);
}

bool lookahead_form(int form) {
    return form == 3 || form == 4 || form == 5 || form == 20 || form == 21 || form == 22 || form == 23;
}

// pass workgroups per band of a publishing form: 256-column tiles (21, 23), 128 (22)
int band_pub_tiles(int form, int64_t width) {
    return (int)(form == 22 ? (width + 127) / 128 : (width + 255) / 256);
}
bool band_pub_ok(const BandPub& bp, const Geometry& g, const Defer& d, int rb) {
    return (d.form == 21 || d.form == 22 || d.form == 23) && d.K == 64 && d.ldc == 64 && rb == bp.rb &&
           (g.rows + rb - 1) / rb <= bp.stride && band_pub_tiles(d.form, g.width) == bp.ntiles &&
           (int64_t)rb * g.ld * 8 < ((int64_t)1 << 31);
}

hipError_t launch_flush_defer(const Geometry& g, const Defer& d, DevState* st, bool nontemporal,
                              int rows_per_block, int occupancy, hipStream_t s, double* Tout,
                              int seal, const BandPub* bp) {
    if (d.K < 1 || d.K > kMaxDefer || rows_per_block < 1 || rows_per_block > 1024 || seal > 1)
        return hipErrorInvalidValue;
    // band publication: lookahead passes of form 21 (band_pub_ok), counted per seal slot
    uint32_t* bcnt = nullptr;
    if (bp && bp->cnt && seal >= 0 && Tout && Tout != g.T && band_pub_ok(*bp, g, d, rows_per_block))
        bcnt = bp->cnt + seal * bp->stride;
    if (g.cd.on) {
        const hipError_t e = launch_reset_cols(g, st, seal, s);
        if (e != hipSuccess) return e;
    }
    return nontemporal ? pass_k<true>(g, d, st, rows_per_block, occupancy, s, Tout, seal, bcnt)
                       : pass_k<false>(g, d, st, rows_per_block, occupancy, s, Tout, seal, bcnt);
}

hipError_t chain_stamps_enable() {
    const int on = 1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_chain_stamps_on), &on, sizeof(on));
}
hipError_t chain_stamps_dump(uint64_t* host64x16) {
    return hipMemcpyFromSymbol(host64x16, HIP_SYMBOL(g_chain_stamps), sizeof(uint64_t) * 64 * 16);
}
hipError_t chain_wg_stamps_dump(uint64_t* host1024x8) {
    return hipMemcpyFromSymbol(host1024x8, HIP_SYMBOL(g_wg_stamps), sizeof(uint64_t) * 1024 * 8);
}

hipError_t launch_reset_cols(const Geometry& g, const DevState* st, int seal, hipStream_t s) {
    if (!g.cd.on || g.rows <= 0) return hipSuccess;
    const int32_t* blkp = seal >= 0 ? &st->seal[seal].blk : &st->blk;
    const int32_t* pl = seal >= 0 ? st->seal[seal].pl : st->pl;
    const int32_t* qs = seal >= 0 ? st->seal[seal].qs : st->qs;
    reset_cols_kernel<<<(unsigned)((g.rows + 255) / 256), 256, 0, s>>>(g.T, g.ld, g.rows, blkp, pl, qs);
    return hipGetLastError();
}

hipError_t launch_seal_defer(DevState* st, int slot, hipStream_t s, const BandPub* bp) {
    if (slot < 0 || slot > 1) return hipErrorInvalidValue;
    seal_kernel<<<1, 64, 0, s>>>(st, slot, bp && bp->cnt ? bp->cnt + slot * bp->stride : nullptr,
                                 bp ? bp->stride : 0);
    return hipGetLastError();
}

}  // namespace dlp
