// dlp_device.h — device-side helpers shared by the pivot kernels
// (dlp_kernels.hip) and the deferred rank-k kernels (dlp_defer.hip):
// pricing / candidate reductions with index tie-breaks, select + pivot log.
// Internal; included inside `namespace dlp { namespace { ... } }`.
#pragma once

typedef double d2 __attribute__((ext_vector_type(2)));
typedef unsigned int u4x __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------- reductions
__device__ inline void pp_combine(PricePart& a, const PricePart& b) {
    if (b.zmin < a.zmin || (b.zmin == a.zmin && b.jmin < a.jmin)) {
        a.zmin = b.zmin;
        a.jmin = b.jmin;
    }
    a.jbland = b.jbland < a.jbland ? b.jbland : a.jbland;
}

__device__ inline PricePart pp_empty() {
    PricePart p;
    p.zmin = __builtin_inf();
    p.jmin = kNoIndex;
    p.jbland = kNoIndex;
    return p;
}

__device__ inline Cand cand_empty() {
    Cand c;
    c.ratio = 0.0;
    c.basis_var = kNoIndex;
    c.row = -1;
    c.valid = 0;
    c.pad0 = 0;
    c.pivot = 0.0;
    return c;
}

// ---- wave-wide minima by DPP (quad permutes, half-row and row mirrors, row broadcasts 15 and
// 31: the minimum lands in lane 63 and is read back uniform): a few cycles per step against the
// LDS round trip of every ds_bpermute a shuffle costs (C5: 6.15 M vs 5.07 M LPs/s, profiles/r04c/).
// Whole waves only; no NaN reaches them (partials and ratios are never NaN: see the callers).
template <int CTRL, int RMASK>
__device__ __forceinline__ double dpp_f64(double v, double id) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v), d = __builtin_bit_cast(uint64_t, id);
    const uint32_t lo = __builtin_amdgcn_update_dpp((int)(uint32_t)d, (int)(uint32_t)u, CTRL, RMASK, 0xf, false);
    const uint32_t hi = __builtin_amdgcn_update_dpp((int)(uint32_t)(d >> 32), (int)(uint32_t)(u >> 32), CTRL, RMASK,
                                                    0xf, false);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, l), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), l);
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
    return readlane_f64(v, 63);
}
template <int CTRL, int RMASK>
__device__ __forceinline__ int32_t dpp_i32(int32_t v) {
    return __builtin_amdgcn_update_dpp(kNoIndex, v, CTRL, RMASK, 0xf, false);
}
__device__ __forceinline__ int32_t wave_min_i32(int32_t v) {
    v = min(v, dpp_i32<0xB1, 0xf>(v));
    v = min(v, dpp_i32<0x4E, 0xf>(v));
    v = min(v, dpp_i32<0x141, 0xf>(v));
    v = min(v, dpp_i32<0x140, 0xf>(v));
    v = min(v, dpp_i32<0x142, 0xa>(v));
    v = min(v, dpp_i32<0x143, 0xc>(v));
    return __builtin_amdgcn_readlane(v, 63);
}

// Wave results of the two reductions, field by field (the same total orders as pp_combine and
// cand_better, so every grouping picks the same winner; uniform results).
// Pricing: min z, the smallest j among the lanes holding it, the smallest Bland j.  (A partial's
// zmin is never NaN: price_pair takes z only when z < zmin.)
__device__ inline PricePart wave_price(const PricePart& v) {
    PricePart o;
    o.zmin = wave_min_f64(v.zmin);
    o.jmin = wave_min_i32(v.zmin == o.zmin ? v.jmin : kNoIndex);
    o.jbland = wave_min_i32(v.jbland);
    return o;
}
// Ratio test: valid first, then the min ratio, then the smallest basis variable (one lane holds
// it: basis variables are distinct).  A valid ratio is never NaN (max(b, 0) / a with a > tol_piv);
// an invalid lane enters as +inf and never ties.
__device__ inline Cand wave_cand(const Cand& c) {
    const double rmin = wave_min_f64(c.valid ? c.ratio : __builtin_inf());
    const bool tie = c.valid && c.ratio == rmin;
    const int32_t bmin = wave_min_i32(tie ? c.basis_var : kNoIndex);
    const uint64_t w = __ballot(tie && c.basis_var == bmin);
    if (w == 0) return cand_empty();
    const int wl = __builtin_amdgcn_readfirstlane(__ffsll((unsigned long long)w) - 1);
    Cand o;
    o.ratio = readlane_f64(c.ratio, wl);
    o.basis_var = __builtin_amdgcn_readlane(c.basis_var, wl);
    o.row = __builtin_amdgcn_readlane(c.row, wl);
    o.valid = 1;
    o.pad0 = 0;
    o.pivot = readlane_f64(c.pivot, wl);
    return o;
}

// Block-wide reduction (whole waves): the wave result, then the waves' results through LDS.
template <typename T, typename Wave, typename Comb>
__device__ inline T block_reduce(T v, T* lds4, Wave wave, Comb comb) {
    v = wave(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) lds4[wid] = v;
    __syncthreads();
    T r = lds4[0];
    const int nw = blockDim.x >> 6;
    for (int w = 1; w < nw; ++w) comb(r, lds4[w]);
    __syncthreads();
    return r;
}

__device__ inline PricePart block_price(PricePart v, PricePart* lds4) {
    return block_reduce(
        v, lds4, [](const PricePart& x) { return wave_price(x); },
        [](PricePart& a, const PricePart& b) { pp_combine(a, b); });
}

__device__ inline Cand block_cand(Cand v, Cand* lds4) {
    return block_reduce(
        v, lds4, [](const Cand& x) { return wave_cand(x); },
        [](Cand& a, const Cand& b) {
            if (cand_better(b, a)) a = b;
        });
}

// Lane-level pricing of two adjacent columns j, j+1 (ascending).
__device__ inline void price_pair(PricePart& acc, double z0, double z1, int64_t j, int64_t ncols,
                                  double tol_dj) {
    if (j < ncols) {
        if (z0 < acc.zmin) { acc.zmin = z0; acc.jmin = (int32_t)j; }
        if (z0 < -tol_dj && acc.jbland == kNoIndex) acc.jbland = (int32_t)j;
    }
    if (j + 1 < ncols) {
        if (z1 < acc.zmin) { acc.zmin = z1; acc.jmin = (int32_t)(j + 1); }
        if (z1 < -tol_dj && acc.jbland == kNoIndex) acc.jbland = (int32_t)(j + 1);
    }
}

// Condensed tableau (Cond): the same for two slots holding variables v0, v1 (-1: not priced), in
// any order: ties to the smaller variable index, Bland's first index = the smallest variable.
__device__ inline void price_pair_var(PricePart& acc, double z0, double z1, int32_t v0, int32_t v1,
                                      double tol_dj) {
    if (v0 >= 0) {
        if (z0 < acc.zmin || (z0 == acc.zmin && v0 < acc.jmin)) { acc.zmin = z0; acc.jmin = v0; }
        if (z0 < -tol_dj && v0 < acc.jbland) acc.jbland = v0;
    }
    if (v1 >= 0) {
        if (z1 < acc.zmin || (z1 == acc.zmin && v1 < acc.jmin)) { acc.zmin = z1; acc.jmin = v1; }
        if (z1 < -tol_dj && v1 < acc.jbland) acc.jbland = v1;
    }
}

// a4: select + basis bookkeeping + pivot log (one lane).
// track: deferred mode, record the step's local pivot row and count it in the block.
// write_obj = false (one-launch pivot): the log entry's objective is left to the commit of the
// same launch, which writes it from another workgroup (the two writes never share bytes).
// cd.on (condensed tableau): the leaving variable takes the entering one's slot st->sq.
__device__ void do_select(DevState* st, const Cand& best, int32_t q, int32_t* basis,
                          int64_t row_first, int64_t rows, int pricing, dlp_pivot* log,
                          int64_t log_cap, bool track = false, bool write_obj = true, Cond cd = Cond{}) {
    if (!best.valid) {
        st->status = DLP_UNBOUNDED;
        return;
    }
    const int32_t p = best.row;
    // the leaving variable: every candidate carries basis[row] (ratio and drive-out kernels), so no
    // dependent load of basis[p] on the selection's critical path
    const int32_t leaving = best.basis_var;
    basis[p] = q;
    st->q = q;
    st->p = p;
    st->leaving = leaving;
    st->ratio = best.ratio;
    st->bland = (pricing == DLP_PRICING_BLAND) ? 1 : (best.ratio == 0.0 ? 1 : 0);
    const int64_t pl = (int64_t)p - row_first;
    st->p_local = (pl >= 0 && pl < rows) ? (int32_t)pl : -1;
    st->piv = best.pivot;
    if (cd.on) {
        const int32_t sq = st->sq;
        cd.slot_of[q] = -1;
        cd.slot_of[leaving] = sq;
        cd.var_of[sq] = leaving;
        if (track) st->qs[st->blk] = sq;
    }
    if (track) {
        st->pl[st->blk] = st->p_local;
        st->blk = st->blk + 1;
    }
    const int64_t k = st->npivots;
    if (log && k < log_cap) {
        if (write_obj) {
            dlp_pivot e;
            e.q = q;
            e.p = p;
            e.leaving = leaving;
            e.pad = 0;
            e.ratio = best.ratio;
            e.objective = __builtin_nan("");
            log[k] = e;
        } else {
            log[k].q = q;
            log[k].p = p;
            log[k].leaving = leaving;
            log[k].pad = 0;
            log[k].ratio = best.ratio;
        }
    }
    st->npivots = k + 1;
}


// ------------------------------------------------------------- peer exchange
// (dlp_internal.h, XPeers).  Every store of a message is a system-scope (sc0 sc1) store into an
// uncached block: written through to its memory, local or across xGMI, and complete once the
// storing wave's vmcnt has drained.  So a message is published by: its stores, every storing
// wave's s_waitcnt vmcnt(0), a workgroup barrier where several waves stored, then ONE flag
// store (the "drained" form: MI355X_MICROARCH.md, inter-workgroup visibility, {sc0 sc1 stores
// and loads both sides}), and read by sc0 sc1 loads after the flag matched.  No release fence:
// on gfx950 a system-scope fence is an L2 write-back + invalidate of the whole XCD L2 (the
// pass's dirty lines included), which the drained form does not need.

__device__ inline void x_store(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ inline uint64_t x_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// This wave's system-scope stores complete (the drained form above).
__device__ inline void x_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
constexpr int kXAux = 1 | 16;   // buffer-op cache policy sc0 sc1 (system scope)
// Bounded wait for *flag == seq: false after xp->wait_ticks (the session's exchange timeout + 5 s;
// 0 = no bound of its own) or when the host raised the abort word.
__device__ inline bool x_wait(const XPeers* xp, const uint64_t* flag, uint64_t seq) {
    if (x_load(flag) == seq) return true;
    const uint64_t t0 = wall_clock64();
    for (uint32_t it = 1;; ++it) {
        __builtin_amdgcn_s_sleep(1);
        if (x_load(flag) == seq) return true;
        if ((it & 255) == 0) {
            if (xp->abort_word &&
                __hip_atomic_load(xp->abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)
                return false;
            if (xp->wait_ticks && wall_clock64() - t0 > xp->wait_ticks) return false;
        }
    }
}
__device__ inline uint64_t* x_cflag(const XPeers* xp, int rank, int parity, int sender, int w = 0) {
    return xp->base[rank] + ((int64_t)parity * xp->nranks + sender) * xp->nslot + w;
}
__device__ inline uint64_t* x_cslot(const XPeers* xp, int rank, int parity, int sender, int w = 0) {
    return xp->base[rank] + xp->off_cslot + (((int64_t)parity * xp->nranks + sender) * xp->nslot + w) * 4;
}
__device__ inline uint64_t* x_rflag(const XPeers* xp, int rank, int64_t chunk) {
    return xp->base[rank] + xp->off_rflag + chunk;
}
__device__ inline uint64_t* x_row(const XPeers* xp, int rank) { return xp->base[rank] + xp->off_row; }

// One lane: a candidate into slot [seq & 1][me][w] of every rank, then the flags.
__device__ inline void x_push_cand(const XPeers* xp, uint32_t seq, const Cand& c, int w = 0) {
    const int par = (int)(seq & 1u);
    const uint64_t* cv = (const uint64_t*)&c;
    for (int r = 0; r < xp->nranks; ++r) {
        uint64_t* slot = x_cslot(xp, r, par, xp->me, w);
#pragma unroll
        for (int k = 0; k < 4; ++k) x_store(slot + k, cv[k]);
    }
    x_drain();   // the slots are complete before any flag
    for (int r = 0; r < xp->nranks; ++r) x_store(x_cflag(xp, r, par, xp->me, w), seq);
}

// Workgroup (xfuse): every rank's ratio-workgroup candidates of exchange seq, reduced in the
// candidate order (any grouping gives the same winner); false when a wait failed.  Lane t takes
// slots t, t + blockDim, ... of the flattened (sender, workgroup) list.
__device__ inline bool x_gather_all(const XPeers* xp, uint32_t seq, Cand* best, int* s_ok) {
    const int par = (int)(seq & 1u);
    if (threadIdx.x == 0) *s_ok = 1;
    __syncthreads();
    Cand b = cand_empty();
    int r = 0, base = 0;   // the sender of slot t: nrat prefix sums, walked forward with t
    for (int t = threadIdx.x;; t += blockDim.x) {
        while (r < xp->nranks && t >= base + xp->nrat[r]) base += xp->nrat[r++];
        if (r >= xp->nranks) break;
        const int w = t - base;
        if (!x_wait(xp, x_cflag(xp, xp->me, par, r, w), seq)) {
            *s_ok = 0;
            break;
        }
        const uint64_t* slot = x_cslot(xp, xp->me, par, r, w);
        Cand o;
        uint64_t* ov = (uint64_t*)&o;
#pragma unroll
        for (int k = 0; k < 4; ++k) ov[k] = x_load(slot + k);
        if (cand_better(o, b)) b = o;
    }
    *best = b;
    __syncthreads();
    return *s_ok != 0;
}

// Workgroup (>= nranks lanes): the P candidates of exchange seq into lds[0..P); false
// when a wait failed (every lane gets the same answer).
__device__ inline bool x_gather_cands(const XPeers* xp, uint32_t seq, Cand* lds, int* s_ok) {
    const int par = (int)(seq & 1u);
    if (threadIdx.x == 0) *s_ok = 1;
    __syncthreads();
    for (int r = threadIdx.x; r < xp->nranks; r += blockDim.x) {
        if (!x_wait(xp, x_cflag(xp, xp->me, par, r), seq)) {
            *s_ok = 0;
            continue;
        }
        const uint64_t* slot = x_cslot(xp, xp->me, par, r);
        uint64_t* dst = (uint64_t*)&lds[r];
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k] = x_load(slot + k);
    }
    __syncthreads();
    return *s_ok != 0;
}

// ---- the selection record (DevState::SelRec): ONE lane publishes, the pivot-row workgroups of
// the same launch wait for it (bounded like every exchange wait)
#ifndef XSEL_SLEEP
#define XSEL_SLEEP 8
#endif
__device__ inline void sel_store32(int32_t* p, int32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void sel_store64(void* p, uint64_t v) {
    __hip_atomic_store((uint64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void sel_publish(DevState* st, uint32_t seq, int32_t status, double zq) {
    DevState::SelRec* r = &st->sel;
    sel_store32(&r->status, status);
    sel_store32(&r->p_local, st->p_local);
    sel_store32(&r->blk, st->blk);
    sel_store64(&r->piv, __builtin_bit_cast(uint64_t, st->piv));
    sel_store64(&r->zq, __builtin_bit_cast(uint64_t, zq));
    sel_store64(&r->npivots, (uint64_t)st->npivots);
    sel_store32(&r->sq, st->sq);
    x_drain();
    __hip_atomic_store(&r->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
struct SelView {
    int32_t status, p_local, blk, sq;
    double piv, zq;
    int64_t npivots;
};
// Workgroup: wait for record seq (lane 0), then every lane gets its fields; false on a failed wait.
__device__ inline bool sel_wait(const XPeers* xp, const DevState* st, uint32_t seq, SelView* out, SelView* lds,
                                int* s_ok) {
    if (threadIdx.x == 0) {
        const DevState::SelRec* r = &st->sel;
        bool ok = __hip_atomic_load(&r->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == seq;
        if (!ok) {
            const uint64_t t0 = wall_clock64();
            for (uint32_t it = 1;; ++it) {
                // (one poller per pivot-row workgroup, ~130 of them on one line: a long sleep keeps
                // the polls from crowding the memory queues the ratio workgroups wait in)
                __builtin_amdgcn_s_sleep(XSEL_SLEEP);
                if (__hip_atomic_load(&r->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == seq) {
                    ok = true;
                    break;
                }
                if ((it & 255) == 0) {
                    if (xp->abort_word &&
                        __hip_atomic_load(xp->abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u)
                        break;
                    if (xp->wait_ticks && wall_clock64() - t0 > xp->wait_ticks) break;
                }
            }
        }
        *s_ok = ok ? 1 : 0;
        if (ok) {
            lds->status = __hip_atomic_load(&r->status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lds->p_local = __hip_atomic_load(&r->p_local, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lds->blk = __hip_atomic_load(&r->blk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lds->sq = __hip_atomic_load(&r->sq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            lds->piv = __builtin_bit_cast(
                double, __hip_atomic_load((const uint64_t*)&r->piv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            lds->zq = __builtin_bit_cast(
                double, __hip_atomic_load((const uint64_t*)&r->zq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            lds->npivots =
                (int64_t)__hip_atomic_load((const uint64_t*)&r->npivots, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    // uniform fields: to SGPRs (the LEAN kernels have 32 VGPRs)
    auto u32 = [](int32_t v) { return (int32_t)__builtin_amdgcn_readfirstlane(v); };
    auto u64 = [](uint64_t v) {
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
        return ((uint64_t)hi << 32) | lo;
    };
    out->status = u32(lds->status);
    out->p_local = u32(lds->p_local);
    out->blk = u32(lds->blk);
    out->sq = u32(lds->sq);
    out->piv = __builtin_bit_cast(double, u64(__builtin_bit_cast(uint64_t, lds->piv)));
    out->zq = __builtin_bit_cast(double, u64(__builtin_bit_cast(uint64_t, lds->zq)));
    out->npivots = (int64_t)u64((uint64_t)lds->npivots);
    const bool ok = u32(*s_ok) != 0;
    __syncthreads();
    return ok;
}

// Workgroup of 256 lanes, chunk = blockIdx.x (512 columns, 2 per lane from column j):
// the owner's row values (v0, v1) into every rank's row region (one 16-B sc0 sc1 store per lane
// and rank; j is even and the region 4 KiB aligned and padded to whole chunks), then, once every
// wave has drained its stores, the chunk flags.
__device__ inline void x_push_row_chunk(const XPeers* xp, uint32_t seq, int64_t j, int64_t ld,
                                        uint64_t v0, uint64_t v1, int chunk) {
    if (j < ld) {
        u4x v;
        v.x = (uint32_t)v0;
        v.y = (uint32_t)(v0 >> 32);
        v.z = (uint32_t)v1;
        v.w = (uint32_t)(v1 >> 32);
        for (int r = 0; r < xp->nranks; ++r) {
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)x_row(xp, r), (short)0, (int)(xp->nchunks * kXChunk * 8), 0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(j * 8), 0, kXAux);
        }
    }
    x_drain();
    __syncthreads();
    for (int r = threadIdx.x; r < xp->nranks; r += blockDim.x) x_store(x_rflag(xp, r, chunk), seq);
}

// Lane j of a chunk (j even): the two row words of this rank's region (one 16-B sc0 sc1 load),
// once the chunk's flag has been seen.
__device__ inline void x_read_row_pair(const XPeers* xp, int64_t j, uint64_t* v0, uint64_t* v1) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)x_row(xp, xp->me), (short)0, (int)(xp->nchunks * kXChunk * 8), 0x00020000);
    const u4x v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(j * 8), 0, kXAux);
    const uint32_t a = v.x, b = v.y, c = v.z, d = v.w;   // (scalars: no element bit-casts)
    *v0 = (uint64_t)a | ((uint64_t)b << 32);
    *v1 = (uint64_t)c | ((uint64_t)d << 32);
}
