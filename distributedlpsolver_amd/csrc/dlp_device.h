// dlp_device.h — device-side helpers shared by the pivot kernels
// (dlp_kernels.hip) and the deferred rank-k kernels (dlp_defer.hip):
// pricing / candidate reductions with index tie-breaks, select + pivot log.
// Internal; included inside `namespace dlp { namespace { ... } }`.
#pragma once

typedef double d2 __attribute__((ext_vector_type(2)));

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

