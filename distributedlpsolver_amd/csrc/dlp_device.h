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

__device__ inline PricePart pp_shfl_xor(const PricePart& v, int m) {
    PricePart o;
    o.zmin = __shfl_xor(v.zmin, m);
    o.jmin = __shfl_xor(v.jmin, m);
    o.jbland = __shfl_xor(v.jbland, m);
    return o;
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

__device__ inline Cand cand_shfl_xor(const Cand& v, int m) {
    Cand o;
    o.ratio = __shfl_xor(v.ratio, m);
    o.basis_var = __shfl_xor(v.basis_var, m);
    o.row = __shfl_xor(v.row, m);
    o.valid = __shfl_xor(v.valid, m);
    o.pad0 = 0;
    o.pivot = __shfl_xor(v.pivot, m);
    return o;
}

// Block-wide reduction (blockDim.x = 256 = 4 waves): wave shuffles, then LDS.
template <typename T, typename Shfl, typename Comb>
__device__ inline T block_reduce(T v, T* lds4, Shfl shfl, Comb comb) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        T o = shfl(v, m);
        comb(v, o);
    }
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
        v, lds4, [](const PricePart& x, int m) { return pp_shfl_xor(x, m); },
        [](PricePart& a, const PricePart& b) { pp_combine(a, b); });
}

__device__ inline Cand block_cand(Cand v, Cand* lds4) {
    return block_reduce(
        v, lds4, [](const Cand& x, int m) { return cand_shfl_xor(x, m); },
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

// a4: select + basis bookkeeping + pivot log (one lane).
// track: deferred mode, record the step's local pivot row and count it in the block.
__device__ void do_select(DevState* st, const Cand& best, int32_t q, int32_t* basis,
                          int64_t row_first, int64_t rows, int pricing, dlp_pivot* log,
                          int64_t log_cap, bool track = false) {
    if (!best.valid) {
        st->status = DLP_UNBOUNDED;
        return;
    }
    const int32_t p = best.row;
    const int32_t leaving = basis[p];
    basis[p] = q;
    st->q = q;
    st->p = p;
    st->leaving = leaving;
    st->ratio = best.ratio;
    st->bland = (pricing == DLP_PRICING_BLAND) ? 1 : (best.ratio == 0.0 ? 1 : 0);
    const int64_t pl = (int64_t)p - row_first;
    st->p_local = (pl >= 0 && pl < rows) ? (int32_t)pl : -1;
    st->piv = best.pivot;
    if (track) {
        st->pl[st->blk] = st->p_local;
        st->blk = st->blk + 1;
    }
    const int64_t k = st->npivots;
    if (log && k < log_cap) {
        dlp_pivot e;
        e.q = q;
        e.p = p;
        e.leaving = leaving;
        e.pad = 0;
        e.ratio = best.ratio;
        e.objective = __builtin_nan("");
        log[k] = e;
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
__device__ inline uint64_t* x_cflag(const XPeers* xp, int rank, int parity, int sender) {
    return xp->base[rank] + (int64_t)parity * xp->nranks + sender;
}
__device__ inline uint64_t* x_cslot(const XPeers* xp, int rank, int parity, int sender) {
    return xp->base[rank] + xp->off_cslot + ((int64_t)parity * xp->nranks + sender) * 4;
}
__device__ inline uint64_t* x_rflag(const XPeers* xp, int rank, int64_t chunk) {
    return xp->base[rank] + xp->off_rflag + chunk;
}
__device__ inline uint64_t* x_row(const XPeers* xp, int rank) { return xp->base[rank] + xp->off_row; }

// One lane: this rank's candidate into slot [seq & 1][me] of every rank, then the flags.
__device__ inline void x_push_cand(const XPeers* xp, uint32_t seq, const Cand& c) {
    const int par = (int)(seq & 1u);
    const uint64_t* cv = (const uint64_t*)&c;
    for (int r = 0; r < xp->nranks; ++r) {
        uint64_t* slot = x_cslot(xp, r, par, xp->me);
#pragma unroll
        for (int k = 0; k < 4; ++k) x_store(slot + k, cv[k]);
    }
    x_drain();   // the slots are complete before any flag
    for (int r = 0; r < xp->nranks; ++r) x_store(x_cflag(xp, r, par, xp->me), seq);
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

// Workgroup of 256 lanes, chunk = blockIdx.x (512 columns, 2 per lane from column j):
// the owner's row values (v0, v1) into every rank's row region (one 16-B sc0 sc1 store per lane
// and rank; j is even and the region 4 KiB aligned and padded to whole chunks), then, once every
// wave has drained its stores, the chunk flags.
__device__ inline void x_push_row_chunk(const XPeers* xp, uint32_t seq, int64_t j, int64_t ld,
                                        uint64_t v0, uint64_t v1) {
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
    for (int r = threadIdx.x; r < xp->nranks; r += blockDim.x) x_store(x_rflag(xp, r, blockIdx.x), seq);
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
