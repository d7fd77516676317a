// dlp_internal.h — types shared by the HIP kernels (dlp_kernels.hip) and the
// host runtime (dlp_session.cpp).  Not part of the public C ABI.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

#include "dlp.h"

namespace dlp {

// Update-kernel geometry: 256 lanes x 2 doubles (one 16-B dwordx4 per lane)
// = one 4 KiB column tile of one tableau row per workgroup-row step.
constexpr int kUpdThreads = 256;
constexpr int kUpdVec = 2;
constexpr int kUpdTile = kUpdThreads * kUpdVec;   // doubles per column tile
constexpr int kRatioThreads = 256;
constexpr int kRatioDeferThreads = 256;  // deferred ratio test (64, 128 and 512 measured slower)
constexpr int kProwThreads = 256;
constexpr int32_t kNoIndex = 0x7fffffff;
constexpr int kColqPad = 16;   // colq allocated with rows + 1 + kColqPad entries
constexpr int32_t kStatusSkip = 5;   // DevState.status: redundant row, forced pivot skipped
constexpr int kMaxDefer = 64;        // deferred rank-k update: at most 64 pivots per tableau pass
constexpr int kMaxReplay = 2 * kMaxDefer;   // steps a selection replays (lookahead: the sealed block + its own)
constexpr int kDeferTile = 512;      // deferred kernels: 256 lanes x 2 doubles per column tile

// Pricing partial of one column tile of the objective row.
struct alignas(16) PricePart {
    double zmin;     // min z_j in the tile (+inf when none)
    int32_t jmin;    // first j attaining zmin (kNoIndex when none)
    int32_t jbland;  // first j with z_j < -tol_dj (kNoIndex when none)
};

// Candidate = dlp_candidate (32 B): ratio, basis_var, row, valid, pad, pivot.
struct alignas(16) Cand {
    double ratio;
    int32_t basis_var;
    int32_t row;
    int32_t valid;
    int32_t pad0;
    double pivot;    // T[row][q] (the pivot element if this row wins)
};
static_assert(sizeof(Cand) == 32, "Cand must match dlp_candidate");

// Device-resident solver state (one per rank).  Every decision of a pivot
// lives here, so a window of pivots runs with no host round trip.
struct alignas(128) DevState {
    int32_t status;    // DLP_RUNNING, DLP_OK (optimal), DLP_UNBOUNDED
    int32_t q;         // entering column
    int32_t p;         // pivot row, global index
    int32_t p_local;   // pivot row on this rank, -1 elsewhere
    int32_t leaving;
    int32_t bland;     // current pricing mode
    int64_t npivots;
    double piv;        // pivot element T[p][q]
    double ratio;      // r_p
    uint32_t ticket;   // last-workgroup election of the ratio kernel
    int32_t blk;       // deferred mode: pivots selected since the last tableau pass
    uint32_t pad[2];
    int32_t pl[kMaxDefer];   // deferred mode: local pivot row of block step l (-1 elsewhere)
    double zq;         // fused deferred pivot: objective-row entry of the entering column
    double pad2[15];
    // fused deferred pivot, on a 128-B line of their own (polled by the pivot-row blocks)
    uint32_t go;       // selection published to the pivot-row blocks
    uint32_t ticket2;  // last pivot-row block re-arms `go`
    uint32_t pad3[30];
    // lookahead (double-buffered tableau): the two most recent sealed blocks, in the
    // layout of (blk, pad, pl) above, so a pass reads either through a BlockDesc*
    struct Seal {
        int32_t blk;
        uint32_t pad[2];
        int32_t pl[kMaxDefer];
        int32_t pad4;
        int32_t ser;              // condensed tableau: the block's serial (bser when sealed)
        int32_t qs[kMaxDefer];    // condensed tableau: slot of each step's entering variable
    } seal[2];
    // peer exchange, one launch per pivot (xfuse 2): the selection handed from the ratio
    // workgroups to the pivot-row workgroups of the same launch, on a line of its own: the fields
    // by sc1 (write-through) stores, drained, then seq (MI355X_MICROARCH.md, first row of the sc1
    // hand-off table); read by sc1 loads after seq matched
    struct alignas(128) SelRec {
        uint32_t seq;
        int32_t status, p_local, blk;
        double piv, zq;
        int64_t npivots;
        int32_t sq;   // condensed tableau: the entering slot
        uint32_t pad[21];
    } sel;
    // condensed tableau (Cond): the entering variable's slot (written with q by the
    // ratio kernel), the open block's serial, and each step's entering slot
    int32_t sq;
    int32_t bser;
    int32_t qs[kMaxDefer];
};
// A pass's block: DevState::blk/pl (in-place passes) or a sealed copy (lookahead).
typedef DevState::Seal BlockDesc;

// Condensed tableau.  A deferred session stores only the columns of the n
// nonbasic variables ("slots" [0, n)) and the RHS (slot n): the m basic columns are exact unit
// vectors (1 in their row, +0 elsewhere; the objective row +0) that the rule never changes, so
// the pass, the pivot-row replay and the exchange move (n + 1) instead of (n + m + 1) columns.
// When variable q (in slot s) enters at row p and v leaves, v takes slot s: its column is the
// step applied to the unit vector e_p, i.e. the replay of slot s restarts at that step from +0
// (row p: the pivot-row rule), and P_step[s] = 1 / pivot.  rst[s] records the restart
// (block serial << 7 | step) for the replays; the pass gets e_p written into its input
// (reset_cols) and P[l < step][s] = +0.  Results, read-outs and pivots are bit-identical to the
// full tableau's (pricing ties by variable index, not slot).
struct Cond {
    int32_t* slot_of = nullptr;   // [N]: slot of a nonbasic variable, -1 for a basic one
    int32_t* var_of = nullptr;    // [ld]: variable in a slot, -1 for the RHS slot and padding
    int32_t* rst = nullptr;       // [ld]: the slot's last restart (serial << 7 | step), -1 none
    int on = 0;
};

// Candidate order: valid first, then smaller ratio, then smaller basis index.
// Total and order-independent, so any reduction tree picks the same winner.
__host__ __device__ inline bool cand_better(const Cand& a, const Cand& b) {
    if (a.valid != b.valid) return a.valid != 0;
    if (!a.valid) return false;
    if (a.ratio != b.ratio) return a.ratio < b.ratio;
    return a.basis_var < b.basis_var;
}

// Peer exchange: the row-block ranks exchange the pivot candidates and the
// owner's pivot row by direct stores into each other's exchange blocks (xGMI peer writes
// between devices; plain stores between sessions on one device), each message followed by
// a tagged flag, instead of an RCCL all-gather + all-reduce.  One block per rank, in
// uncached device memory, laid out identically on every rank (uint64 words):
//   [0, 2PS)                   candidate flags  cflag[parity][sender][w]  (= exchange seq)
//   [off_cslot, +8PS)          candidate slots  cslot[parity][sender][w]  (4 words = 32 B)
// with S = nslot slots per sender: slot w = 0 carries the rank's candidate (the select kernel's
// exchange), or, when the ratio launch selects (xfuse), w = the ratio workgroup: every workgroup
// pushes its own candidate and workgroup 0 of every rank reduces all of them (no ticket).
//   [off_rflag, +nchunks)      pivot-row chunk flags (512 columns per chunk)
//   [off_row, +ld)             the pivot row (fp64 bits), written by its owner
// Every wait is bounded (wait_ticks of the 100 MHz constant clock: the host's exchange timeout
// + 5 s, 0 = none; and the host's abort word): a stall sets DevState.status = kStatusXFail and
// the host returns DLP_ERR_RCCL, as for every exchange failure.
constexpr int kMaxRanks = 64;
constexpr int kXChunk = 512;                       // pivot-row chunk (= prow / commit workgroup)
constexpr int32_t kStatusXFail = 6;                // DevState.status: a peer exchange timed out
struct XPeers {
    uint64_t* base[kMaxRanks];   // every rank's exchange block as this device addresses it
    const uint32_t* abort_word;  // host-pinned; nonzero ends every wait (dlp_session_abort)
    int32_t nranks, me;
    uint64_t wait_ticks;         // bound of one wait (0: the abort word only)
    int64_t nchunks;
    int64_t off_cslot, off_rflag, off_row;
    int32_t nslot;               // candidate slots per sender (>= every rank's ratio workgroups)
    int32_t nrat[kMaxRanks];     // ratio workgroups of each rank (its candidates under xfuse)
};
// Block size (bytes) and offsets for nranks ranks, row length ld and nslot slots per sender.
size_t xblock_layout(int nranks, int64_t ld, int nslot, XPeers* xp);

// Deferred rank-k update (dlp_defer.hip).  Up to K pivots are selected against
// the stale HBM tableau T0 through "replayed" views (column q and pivot row p
// re-derived by applying the block's earlier steps, in order, with the same
// fma / overwrite / skip per element as the eager update); the objective row
// and the RHS column are kept current eagerly; one pass then applies all
// steps to every element in order.  Every value is therefore bit-identical to
// K eager rank-1 updates while the tableau is streamed once per K pivots.
struct Defer {
    int K = 1;             // block size (1 = eager path, no deferral)
    double* C = nullptr;   // (rows+1) x K row-major: C[i*ldc + l] = T_l[i][q_l]
    int64_t ldc = 0;       // = K (row `rows` = the objective row's entries)
    double* Cc = nullptr;  // K x ldcc column-major copy of C: Cc[l*ldcc + i] (the ratio
    int64_t ldcc = 0;      // kernel's replay loads, coalesced); ldcc = round64(rows + 1)
    double* P = nullptr;   // K x ld: normalised pivot rows
    double* rhs = nullptr; // rows: current RHS column (eager cache)
    int32_t* nzc = nullptr; // rows: nonzero C[i][l] of the block so far (the pass's row class)
    int form = 3;          // pass kernel, LDS-staged coefficients: 0 = 2 doubles/lane,
                           // 1 = 1 double/lane x 2 rows, 2 = 1 double/lane x 4 rows;
                           // scalar-coefficient forms: 3 = 1 double x 4 rows (default; 4 at K = 32 streaming),
                           // 4 = 2 doubles x 2 rows, 5 = 1 double x 8 rows
};

// Lookahead band publication: the form-21 pass of seal slot s counts its
// finished workgroups per band in cnt[s * stride + band]; a band whose count reached ntiles
// is final in Tn, so the next block's selections read its rows there and replay only their
// own block (bit-identical: the pass computes the same operations in the same order).
struct BandPub {
    uint32_t* cnt = nullptr;    // [2][stride]
    int64_t stride = 0;         // >= the pass's bands
    int rb = 0;                 // pass rows per band
    int ntiles = 0;             // pass workgroups per band (band_pub_tiles)
    const double* Tn = nullptr; // the pass's output buffer (set per pass by the session)
};
struct Geometry;
bool band_pub_ok(const BandPub& bp, const Geometry& g, const struct Defer& d, int rb);
int band_pub_tiles(int form, int64_t width);

static_assert(offsetof(DevState, pl) - offsetof(DevState, blk) == offsetof(BlockDesc, pl),
              "BlockDesc must alias DevState::blk / pl");

// Launchers (dlp_kernels.hip).  All asynchronous on `stream`.
struct Geometry {
    double* T;            // (rows+1) x ld, objective row last
    int64_t ld;           // row stride (>= width, multiple of ld_align)
    int64_t width;        // round16(N+1): columns the kernels touch
    int64_t rows;         // local constraint rows
    int64_t row_first;    // global index of local row 0
    int64_t ncols;        // N (RHS column index): n + m, or the general LP's total columns
    int64_t nprice;       // columns [0, nprice) are priced (general LPs: artificials excluded)
    int64_t rows_elig;    // local rows [0, rows_elig) take part in the ratio test (the
                          // carried Phase II objective row, when present, is local row rows-1)
    int ntiles;           // ceil(ld / kUpdTile)
    int rows_per_block;   // update kernel
    int rthreads = kRatioDeferThreads;   // deferred ratio workgroup (64 / 128 / 256 lanes; the
                                         // session's ratio_threads_policy, fixed at creation)
    Cond cd;              // condensed tableau (cd.on): ncols = n is the RHS slot, width = round16(n + 1)
};

// Update-kernel variants (tuning): 0 U4/2dbl/scalar-colq (default), 1 U8, 2 U4/LDS-colq,
// 3 U8/LDS, 4 U4/4dbl, 5 U2/4dbl, 6 U4/4dbl/LDS, 7 U16/LDS.  Column tile = update_tile().
int update_tile(int variant);
int update_variants();
constexpr int kMaxBandLdsHost = 256;   // LDS-colq variants need rows_per_block <= this
hipError_t launch_price_init(const Geometry& g, PricePart* pp, double tol_dj, int variant,
                             hipStream_t s);
hipError_t launch_ratio(const Geometry& g, const int32_t* basis_in, int32_t* basis_out,
                        const PricePart* pp, DevState* st, double* colq, Cand* partials,
                        int nblocks, Cand* cand_out, int nranks, double tol_dj, double tol_piv,
                        int pricing, dlp_pivot* log, int64_t log_cap, hipStream_t s);
// Peer exchange kernels (dlp_kernels.hip).  xcand_send: this rank's candidate (cand_send)
// into every rank's slot (seq); the select kernel waits for and reduces the P slots when
// given xp.  xrow_send: the owner's pivot-row bits (owner: st->p_local >= 0, or
// owner_rank >= 0 for the carried row) into every rank's row region + chunk flags;
// xrow_recv: wait for every chunk of this seq and copy the row to `out` (a plain buffer
// for the eager kernels).
hipError_t launch_xcand_send(const XPeers* xp, uint32_t seq, const Cand* cand_send, const DevState* st,
                             hipStream_t s);
hipError_t launch_xwait(const XPeers* xp, uint32_t seq, DevState* st, hipStream_t s);
hipError_t launch_xrow_send(const XPeers* xp, uint32_t seq, const int64_t* bits, int64_t ld,
                            const DevState* st, int owner_rank, int my_rank, hipStream_t s);
hipError_t launch_xrow_recv(const XPeers* xp, uint32_t seq, int64_t ld, int64_t* out, DevState* st,
                            hipStream_t s);
int ratio_blocks(const Geometry& g);
int ratio_defer_blocks(const Geometry& g);
hipError_t launch_select(const Geometry& g, const Cand* cands, int nranks, int32_t* basis,
                         DevState* st, int pricing, dlp_pivot* log, int64_t log_cap,
                         hipStream_t s, bool forced = false, bool track = false,
                         const XPeers* xp = nullptr, uint32_t seq = 0);
// Condensed tableau: the initial slot maps (variables 0..n-1 in slots 0..n-1, the m slacks basic),
// no restarts; and the block's restart columns e_p written into the pass input (before its pass).
hipError_t launch_cond_init(const Geometry& g, int64_t N, DevState* st, hipStream_t s);
hipError_t launch_reset_cols(const Geometry& g, const DevState* st, int seal, hipStream_t s);
// General LPs (Phase I -> II).  drive: forced-pivot candidate for global row
// `row` (nranks == 1: also select + colq capture); gather_q: colq of st->q;
// carry_out / carry_in: ship the carried objective row through the int64 MAX
// exchange buffers and install it as the objective row (status -> running).
hipError_t launch_drive(const Geometry& g, int64_t row, int32_t* basis, DevState* st,
                        double tol_piv, Cand* cand_out, int nranks, int pricing, dlp_pivot* log,
                        int64_t log_cap, double* colq, hipStream_t s);
hipError_t launch_gather_q(const Geometry& g, const DevState* st, double* colq, hipStream_t s);
hipError_t launch_carry_out(const Geometry& g, int64_t carry_local, int64_t* out, hipStream_t s);
hipError_t launch_carry_in(const Geometry& g, const int64_t* in, DevState* st, int pricing,
                           hipStream_t s);
hipError_t launch_set_status(DevState* st, int status, hipStream_t s);

// Deferred launchers (dlp_defer.hip).  Pricing tiles are kDeferTile columns.
// prev / prev_seal (lookahead): the sealed block st->seal[prev_seal] whose arrays are
// `prev` is not yet applied to g.T; its steps are replayed before the current block's.
// bp (lookahead at K = 64): the pass in flight publishes its finished bands (BandPub).
hipError_t launch_ratio_defer(const Geometry& g, const Defer& d, int32_t* basis,
                              const PricePart* pp, DevState* st, Cand* partials, int nblocks,
                              Cand* cand_out, int nranks, double tol_dj, double tol_piv,
                              int pricing, dlp_pivot* log, int64_t log_cap, hipStream_t s,
                              const Defer* prev = nullptr, int prev_seal = -1,
                              const XPeers* xp = nullptr, uint32_t seq = 0, const BandPub* bp = nullptr,
                              bool xfuse = false, bool own_cus = false);
// xfuse (peer exchange, nranks > 1): the last workgroup also waits for every rank's candidate and
// selects (no select launch); launch_prow_defer's xfuse: the pivot-row launch also commits the
// exchanged row (no commit launch).  Only where each rank's launches run on hardware queues of
// their own (one rank per device or process): a wait inside a launch is then never queued behind
// the launch of another rank that it waits for (dlp_sessions_run of ranks sharing a device does not
// fuse).
// Peer exchange (xfuse sessions), ONE launch per pivot: the ratio test, the candidates of every
// workgroup to every rank, the selection by workgroup 0, its record to the pivot-row workgroups of
// the same launch, the owner's row push and every rank's commit.
hipError_t launch_pivot_x(const Geometry& g, const Defer& d, int32_t* basis, PricePart* pp, DevState* st,
                          double tol_dj, double tol_piv, int pricing, dlp_pivot* log, int64_t log_cap,
                          hipStream_t s, const Defer* prev, int prev_seal, const XPeers* xp, uint32_t seq,
                          const BandPub* bp, bool own_cus = false);
// nranks == 1: ratio test + selection + pivot row + objective row + pricing in ONE launch
// (K <= 32; grid of fused_pivot_blocks(g), all of which must be resident at once).
int fused_pivot_blocks(const Geometry& g);
int fused_pivot_capacity(int K, int cus);   // resident workgroups of the fused kernel (0: unknown)
hipError_t launch_pivot_defer(const Geometry& g, const Defer& d, int32_t* basis, PricePart* pp,
                              DevState* st, Cand* partials, int nblocks, double tol_dj,
                              double tol_piv, int pricing, dlp_pivot* log, int64_t log_cap,
                              hipStream_t s);
// nranks == 1: P[s] + objective row + pricing partials + log in one pass;
// nranks > 1: the owner's replayed pivot-row bits (others INT64_MIN) to prow_bits.
// xp (peer exchange): the owner stores its row into every rank's row region + chunk
// flags instead (non-owners write nothing).
hipError_t launch_prow_defer(const Geometry& g, const Defer& d, const DevState* st,
                             int64_t* prow_bits, PricePart* pp, double tol_dj, dlp_pivot* log,
                             int64_t log_cap, int nranks, hipStream_t s,
                             const Defer* prev = nullptr, int prev_seal = -1,
                             const XPeers* xp = nullptr, uint32_t seq = 0, const BandPub* bp = nullptr,
                             bool xfuse = false, bool own_cus = false);
// nranks > 1, after the MAX all-reduce: P[s] from the exchanged bits + objective row + pricing.
// xp: each workgroup first waits for its chunk's flag (seq), then reads the row region
// with system-scope loads (prow_bits = this rank's row region).
hipError_t launch_commit_defer(const Geometry& g, const Defer& d, DevState* st,
                               const int64_t* prow_bits, PricePart* pp, double tol_dj,
                               dlp_pivot* log, int64_t log_cap, hipStream_t s,
                               const XPeers* xp = nullptr, uint32_t seq = 0);
// The tableau pass: applies the block's st->blk steps to rows [0, rows), then blk = 0.
// Lookahead (seal >= 0): the block st->seal[seal], read from g.T and written to Tout
// (every row, untouched ones copied; blk is left alone).  Only the forms with an
// out-of-place instance: lookahead_form() is the single source of truth (3, 4, 5, 20, 21,
// 22, 23).
hipError_t launch_flush_defer(const Geometry& g, const Defer& d, DevState* st, bool nontemporal,
                              int rows_per_block, int occupancy, hipStream_t s,
                              double* Tout = nullptr, int seal = -1, const BandPub* bp = nullptr);
bool lookahead_form(int form);
// Diagnostics (DLP_CHAIN_STAMPS): phase stamps of the LEAN chain kernels (dlp_defer.hip).
hipError_t chain_stamps_enable();
hipError_t chain_stamps_dump(uint64_t* host64x16);
hipError_t chain_wg_stamps_dump(uint64_t* host1024x8);
// End of a lookahead block: st->seal[slot] := (blk, pl), blk := 0.
hipError_t launch_seal_defer(DevState* st, int slot, hipStream_t s, const BandPub* bp = nullptr);
hipError_t launch_prow(const Geometry& g, const DevState* st, int64_t* prow_bits, int nranks,
                       hipStream_t s);
hipError_t launch_update(const Geometry& g, const double* colq, const double* prow,
                         const DevState* st, PricePart* pp, double tol_dj, dlp_pivot* log,
                         int64_t log_cap, bool nontemporal, int variant, hipStream_t s);
// Small LPs: the tableau in the LDS of nwg workgroups (cluster_plan; 0 = does not
// fit), `max_pivots` pivots of the eager rule per launch (dlp_cluster.hip).
size_t cluster_lds_bytes(int64_t m, int cw);
int cluster_plan(int64_t m, int64_t N, int max_wg, int* cw_out);
int64_t cluster_gstride(int64_t m);
int64_t cluster_granules(int64_t m, int nwg);   // uint64 hand-off words of a launch
hipError_t launch_cluster(const Geometry& g, int64_t m, int64_t n, int nwg, int cw, DevState* st,
                          int32_t* basis, dlp_pivot* log, int64_t log_cap, uint64_t* gran,
                          int64_t max_pivots, int pricing, double tol_dj, double tol_piv,
                          hipStream_t s, uint64_t* stamps = nullptr);
// Synthetic tableau rows [row_first, row_first+rows) + objective row, on device.
hipError_t launch_generate(const Geometry& g, int kind, int64_t m, int64_t n, uint64_t seed,
                           hipStream_t s);
// Gather column `col` of rows [0, nrows) into out (nrows doubles).
hipError_t launch_gather_column(const double* T, int64_t ld, int64_t nrows, int64_t col,
                                double* out, hipStream_t s);

// dlp_batched.hip: free the cached dlp_batched_solve contexts of `device` (-1: all); bytes freed
size_t batched_release(int device);

}  // namespace dlp
