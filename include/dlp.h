/*
 * dlp.h — C ABI of the MI355X-native dense-tableau fp64 simplex (libdlp.so).
 *
 * This is the drop-in boundary for the per-iteration solver core of
 * shidanxu/DistributedLPSolver.  The reference has no FFI:
 * its surface is in-process C++ (namespace distributed_solver).  Each entry
 * point below names the reference interface it replaces; R/ is
 * /root/reference/DistributedLPSolver/DistributedLPSolver/.
 *
 *   reference                                         this ABI
 *   ------------------------------------------------  ---------------------------------
 *   Instance::Instance(A, I, slots, sparsity, ...)     dlp_problem_create_adalloc
 *     R/instance.h:41-42, R/instance.cpp:15-30
 *   Instance::GenerateInstance()  R/instance.h:46      dlp_problem_create_adalloc (bids
 *     R/instance.cpp:32-57                             regenerated bit-exactly, glibc rand)
 *   (no reference: dense LP input)                     dlp_problem_create_dense / _random
 *   Instance::RunMultiplicativeWeights(...)            dlp_solve  (exact simplex instead of
 *     R/instance.h:52-53, R/instance.cpp:117-134       the epsilon-approximate MW loop)
 *   GlobalProblem::ConstructPrimal per-iteration core  dlp_session_step_* (one pivot)
 *     R/global_problem.cpp:257-323                     dlp_session_run   (K pivots)
 *   Instance::solution_ (private, no getter)           dlp_result_x / dlp_result_y
 *     R/instance.h:34
 *   "Dual Value" stdout  R/global_problem.cpp:320-322  dlp_result_objective
 *
 * Conventions (build conventions):
 *   - every function returns int status: DLP_OK (0) or a code below; no C++
 *     exception ever crosses this boundary;
 *   - the library owns problems, sessions and results; the caller frees them
 *     with the matching *_free;
 *   - a handle is not thread-safe; concurrent solves on distinct handles are;
 *   - all arrays are plain host pointers unless the name says "dev";
 *   - fp64 everywhere (the reference computes in x87 long double; see DESIGN.md
 *     for what "parity" therefore means).
 *
 * Pivot rule (identical in oracle/ and on the GPU):
 *   maximise c^T x  s.t.  A x <= b, x >= 0, b >= 0, slack starting basis.
 *   Tableau T is (m+1) x (N+1), N = n + m, row-major, leading dimension
 *   ld = roundup(N+1, 16); row m is the objective (z_j, initially -c_j).
 *   price   : Dantzig q = argmin_{j<N} z_j (ties -> smallest j), optimal when
 *             z_q >= -tol_dj; in Bland mode q = smallest j with z_j < -tol_dj.
 *             Bland mode is entered after a degenerate pivot (r_p == 0) and
 *             left after a non-degenerate one (DLP_PRICING_DANTZIG_BLAND), or
 *             always on (DLP_PRICING_BLAND).
 *   ratio   : rows i<m with T[i][q] > tol_piv; r_i = max(T[i][N],0) / T[i][q]
 *             (IEEE division); p = argmin r_i, exact ties -> smallest basis[i];
 *             unbounded when no row qualifies.
 *   update  : prow_j = T[p][j] / T[p][q]; for i != p with T[i][q] != 0:
 *             T[i][j] = fma(-T[i][q], prow_j, T[i][j]); row p := prow; rows with
 *             T[i][q] == 0 are left untouched.
 */
#ifndef DLP_H
#define DLP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---------------------------------------------------- */
#define DLP_OK              0   /* optimal (or the step/run completed) */
#define DLP_INFEASIBLE      1   /* general LPs: Phase I ended with artificials > tol_feas */
#define DLP_UNBOUNDED       2
#define DLP_PIVOT_LIMIT     3
#define DLP_RUNNING         4   /* session has pivots left to do */
#define DLP_ERR_ARG        -1
#define DLP_ERR_OOM        -2
#define DLP_ERR_HIP        -3
#define DLP_ERR_RCCL       -4
#define DLP_ERR_NODEVICE   -5
#define DLP_ERR_STATE      -6
#define DLP_ERR_UNSUPPORTED -7

/* ---- enums ------------------------------------------------------------ */
#define DLP_PRICING_DANTZIG_BLAND 0
#define DLP_PRICING_BLAND         1

/* Synthetic instance families. */
#define DLP_GEN_DENSE       0   /* A,x0,c ~ U[0,1); b = A x0 + U[0,1)          */
#define DLP_GEN_DEGENERATE  1   /* ~50% "cone" rows: A in [-1,1), b_i = 0      */

/* Exchange buffers of a rank session (dlp_session_buffer). */
#define DLP_BUF_CAND_SEND   0   /* 1 x dlp_candidate, device                   */
#define DLP_BUF_CAND_RECV   1   /* nranks x dlp_candidate, device              */
#define DLP_BUF_PROW_SEND   2   /* ld x int64 (fp64 bits or INT64_MIN), device */
#define DLP_BUF_PROW_RECV   3   /* ld x int64, device                          */

/* Timing phases (dlp_session_timings, milliseconds, HIP events). */
#define DLP_PHASE_RATIO     0   /* pricing reduce + ratio test kernel          */
#define DLP_PHASE_EXCHANGE  1   /* candidate all-gather + select (nranks > 1)  */
#define DLP_PHASE_PROW      2   /* pivot-row normalise (+ all-reduce)          */
#define DLP_PHASE_UPDATE    3   /* rank-1 elimination kernel                   */
#define DLP_NUM_PHASES      4

typedef struct dlp_problem dlp_problem;
typedef struct dlp_session dlp_session;
typedef struct dlp_result  dlp_result;

/* 32-byte ratio-test candidate exchanged between ranks (all-gather). */
typedef struct dlp_candidate {
    double  ratio;      /* r_i */
    int32_t basis_var;  /* basis[i] (tie-break) */
    int32_t row;        /* global row index */
    int32_t valid;      /* 0 = no eligible row on that rank */
    int32_t pad0;
    double  pivot;      /* T[row][q], the pivot element if this row wins */
} dlp_candidate;

/* 32-byte pivot-log entry: the parity artifact. */
typedef struct dlp_pivot {
    int32_t q;          /* entering column */
    int32_t p;          /* pivot row (global) */
    int32_t leaving;    /* basis[p] before the pivot */
    int32_t pad;
    double  ratio;      /* r_p */
    double  objective;  /* T[m][N] after the pivot */
} dlp_pivot;

typedef struct dlp_options {
    int32_t device;          /* HIP device ordinal (default 0) */
    int32_t pricing;         /* DLP_PRICING_* */
    double  tol_dj;          /* reduced-cost tolerance (default 1e-9) */
    double  tol_piv;         /* pivot-element tolerance (default 1e-9) */
    int64_t max_pivots;      /* pivot limit (default 1000000) */
    int32_t log_pivots;      /* keep the pivot log (default 1) */
    int32_t check_interval;  /* pivots between host status polls (default 64) */
    int32_t timing;          /* 0 none, 1 update kernel, 2 every phase */
    int32_t nontemporal;     /* update kernel nt loads/stores: 1/0, -1 = auto (default) */
    int32_t rows_per_block;  /* update-kernel rows per workgroup band (0 = auto, default) */
    int32_t use_graph;       /* replay each poll window as a hipGraph (default 1) */
    int32_t update_variant;  /* rank-1 kernel variant 0..dlp_update_variants()-1, -1 = auto (default) */
    int32_t ld_align;        /* tableau row stride alignment in doubles, multiple of 16, 0 = auto
                                (default: when a row has >= 4096 columns, 128 for a deferred
                                session on a tableau > 1 GiB and 512 otherwise; else 16); the
                                kernels only touch the first roundup(N+1,16) columns */
    int32_t small_lp;        /* one-launch LDS solve for small LPs (dlp_cluster.hip): 0 = auto
                                (default: single-rank dense / random / ad-allocation problems
                                whose tableau is under 32 MiB and fits the LDS of the device's
                                CUs), 1 = whenever it fits, -1 = never */
    double  tol_feas;        /* general LPs: infeasible when the Phase I optimum is below
                                -tol_feas * (1 + max_i b'_i) (default 1e-9) */
    int32_t defer;           /* pivots per tableau pass (deferred rank-k update, results
                                bit-identical to rank-1): 1 = eager rank-1 per pivot, 2..64 =
                                block size, 0 = auto (default: 64 on a tableau > 1 GiB, 16
                                from 32 MiB, eager below 32 MiB and for multi-rank sessions
                                without an RCCL id, whose exchange the caller drives
                                through dlp_session_step_*; a single-rank session driven
                                through the step API keeps the size-based choice) */
    int32_t n_gpus;          /* dlp_solve only: 0 (default) = one GPU, no communicator;
                                N >= 1 = a row-block solve on devices [device, device+N) of
                                this process: one host thread and one RCCL communicator
                                rank per device (ncclCommInitAll); N = 1 runs that path on
                                a 1-rank communicator.  Sessions ignore it (one process per
                                GPU: dlp_session_create_rank). */
    int32_t lookahead;       /* deferred sessions: select block b+1 while the pass of block b
                                runs, on a second tableau buffer (results unchanged, bit for
                                bit; 2x the tableau memory): 1 = on where supported, 0 = off,
                                -1 = auto (default: K = 64 on a streaming (> 1 GiB) tableau
                                that fits twice, single-rank or a row-block rank once it runs
                                the peer exchange, never with RCCL; at K = 64 the selections
                                replay up to 127 steps) */
    int32_t exchange;        /* row-block exchange of dlp_solve(n_gpus = N) and of rank sessions
                                created with an RCCL id: DLP_XCHG_DEFAULT (0, the default) = the
                                peer exchange where every rank pair connects (peer access + IPC
                                open, agreed by all ranks), else RCCL (the reason:
                                dlp_session_exchange_reason); DLP_XCHG_RCCL = RCCL candidate
                                all-gather + pivot-row MAX all-reduce; DLP_XCHG_PEER = owner-
                                rooted peer stores, an error when the ranks cannot connect.
                                dlp_solve(n_gpus) with DLP_XCHG_DEFAULT: a run that fails on the
                                peer exchange is rerun from the start over RCCL
                                (dlp_result_exchange reports it) */
    int32_t condensed;       /* deferred sessions (defer > 1) of dense / random / ad-allocation LPs:
                                store only the n nonbasic columns + the RHS, the m basic columns
                                being exact unit vectors (results, pivots and
                                read-outs bit-identical to the full tableau): 1 = on where
                                supported, -1 = off, 0 = auto (default: on; DLP_CONDENSED=0/1
                                overrides auto) */
} dlp_options;
/* Auto tuning (MI355X measurements): a local tableau > 1 GiB streams
 * from HBM -> row-serial kernel capped at 4 workgroups/CU, 8-row bands, nt;
 * otherwise it is partly Infinity-Cache resident -> uncapped, 4-row bands. */

/* ---- library ---------------------------------------------------------- */
void        dlp_options_default(dlp_options* opt);
const char* dlp_status_string(int status);
const char* dlp_last_error(void);          /* thread-local message of the last failure */
int         dlp_device_count(int* count);
/* Row partition of m constraint rows over nranks: [first, first+count). */
int         dlp_rank_rows(int64_t m, int rank, int nranks, int64_t* first, int64_t* count);
/* Deterministic winner of nranks candidates (same rule as the device select). */
int         dlp_candidate_select(const dlp_candidate* cands, int n, int* winner);
int64_t     dlp_tableau_ld(int64_t m, int64_t n);   /* roundup(N+1,16); sessions may pad more */
int         dlp_update_variants(void);               /* number of rank-1 update variants */
/* Sessions return their small buffers (<= 32 MiB each, <= 512 MiB in all) and streams to a
 * per-process cache for the next session, and dlp_batched_solve keeps one context per device
 * (stream, events, tableau / output buffers sized by the largest batch so far).  This frees the
 * cached buffers, pooled streams and batch contexts of `device` (-1: every device and the pinned host
 * buffers);
 * *bytes (may be NULL) = device bytes freed.  A session allocation that fails frees its device's
 * cached session buffers and retries by itself; that hipFree may synchronise the device, so it
 * waits for work other sessions have in flight on it (call this between runs to avoid that). */
int         dlp_release_cached_memory(int device, int64_t* bytes);

/* ---- problems ------------------------------------------------------------ */
/* Dense LP: A is m x n row-major; inputs are copied. Requires b >= 0. */
int dlp_problem_create_dense(int64_t m, int64_t n, const double* A, const double* b,
                             const double* c, dlp_problem** out);
/* Synthetic LP generated on the device (no host copy of A). */
int dlp_problem_create_random(int kind, int64_t m, int64_t n, uint64_t seed, dlp_problem** out);
/* The reference's ad-allocation LP (R/instance.cpp:32-57, R/allocation_mw.cpp:163-171):
 * max sum b_ai x_ai  s.t.  sum_i b_ai x_ai <= B_a (A rows),  sum_a x_ai <= 1 (I rows). */
int dlp_problem_create_adalloc(int num_advertisers, int num_impressions, int num_slots,
                               double bid_sparsity, double scaling_factor, dlp_problem** out);
/* ---- general LPs: row/column bounds + two-phase -------
 *   minimise (sense = DLP_MINIMIZE) or maximise (DLP_MAXIMIZE)  c^T x + c0
 *   s.t.  row_lo <= A x <= row_hi,  col_lo <= x <= col_hi,
 * A dense m x n row-major; any bound may be infinite (|v| >= 1e30 counts as
 * infinite).  No reference interface: the reference only builds its own
 * ad-allocation LP in memory (R/instance.cpp:32-57).  Netlib-style inputs come
 * through dlp_problem_create_mps.
 *
 * Canonical standard form (the rule spec; oracle/oracle.cpp restates it):
 *  columns: user variable j in order -> lo finite: x_j = lo + x' (one column;
 *           plus a bound row x' <= hi - lo when hi is finite); lo = -inf, hi
 *           finite: x_j = hi - x' (column -A_j, cost -c_j); both infinite:
 *           x_j = x'+ - x'- (two adjacent columns +A_j, -A_j).
 *  rows:    user rows in order, then the bound rows in column order.  shift_i
 *           = fma-chain over j ascending of A_ij * const_j (const = lo or hi).
 *           lo == hi -> E row (rhs lo - shift); only hi finite -> L row; only lo
 *           finite -> G row; both finite -> L row (hi) then G row (lo); both
 *           infinite -> dropped.  A row with rhs < 0 is negated (L <-> G); a G
 *           row with rhs == 0 is negated into an L row; rhs -0.0 becomes +0.0.
 *  tableau: [structural | one slack (+1, L) / surplus (-1, G) column per L/G
 *           row, in row order | one artificial (+1) column per G/E row, in row
 *           order | RHS].  Pricing covers structural + slack/surplus columns
 *           only (artificials never enter).  Basis: slack of L rows,
 *           artificial of G/E rows.  Objective (max form) c' = -c for minimise.
 *  phase I  (only when there are artificials): objective row z_j = sum over
 *           artificial rows i ascending of (-T[i][j]) for every non-artificial
 *           column j and the RHS (left fold from 0.0, z_j - T[i][j]); the
 *           phase II objective (-c', 0 elsewhere) rides along as an extra
 *           tableau row (global row m', owned by the last rank, never in the
 *           ratio test).  Pivot rule exactly as above.  At the Phase I optimum:
 *           infeasible if z_N < -tol_feas (1 + max b'); else every row whose
 *           basic variable is artificial, ascending, is pivoted on its first
 *           column q < n_price with |T[i][q]| > tol_piv (a logged pivot with
 *           ratio 0; a row without one is redundant and keeps its artificial);
 *           then the carried row becomes the objective row and Phase II runs
 *           in the pricing mode of the options (Bland state reset).
 *  results: x in user variables; y[i] = d(user objective)/d(bound of user row
 *           i) (HiGHS / scipy "marginals" sign convention), summed over the
 *           two rows of a ranged row; objective in the user's sense incl. c0. */
#define DLP_MINIMIZE   1
#define DLP_MAXIMIZE  -1
int dlp_problem_create_general(int64_t m, int64_t n, const double* A, const double* row_lo,
                               const double* row_hi, const double* col_lo, const double* col_hi,
                               const double* c, double c0, int sense, dlp_problem** out);
/* Free- or fixed-format MPS file (whitespace-separated fields; names without
 * blanks): NAME, OBJSENSE (MIN/MAX), ROWS (N/L/G/E; the first N row is the
 * objective, later N rows are dropped), COLUMNS (MARKER lines ignored: integer
 * columns are relaxed; repeated entries are summed), RHS (an objective-row RHS
 * v sets c0 = -v), RANGES (standard L/G/E semantics), BOUNDS (UP LO FX FR MI
 * PL BV LI UI; UP < 0 with lower 0 sets lower = -inf), ENDATA. */
int dlp_problem_create_mps(const char* path, dlp_problem** out);
/* The general form of any non-random problem (arrays may be NULL). */
int dlp_problem_get_general(const dlp_problem* prob, double* A, double* row_lo, double* row_hi,
                            double* col_lo, double* col_hi, double* c, double* c0, int* sense);
/* Standard-form sizes: constraint rows m' (the tableau adds the carried row
 * when nart > 0), total columns N, priced columns, artificial columns.  For
 * dense / random / ad-allocation problems: m' = m, N = n_price = n + m, 0. */
int dlp_problem_std_dims(const dlp_problem* prob, int64_t* m_std, int64_t* ncols,
                         int64_t* nprice, int64_t* nart);

int dlp_problem_dims(const dlp_problem* prob, int64_t* m, int64_t* n);
/* Dense copy of the problem data (A m x n row-major, b, c); NULL pointers skipped. */
int dlp_problem_get_dense(const dlp_problem* prob, double* A, double* b, double* c);
/* Ad-allocation bid list in variable order: (advertiser, impression, bid) triples. */
int dlp_problem_adalloc_bids(const dlp_problem* prob, int64_t* nnz, int32_t* adv,
                             int32_t* imp, double* bid);
void dlp_problem_free(dlp_problem* prob);

/* ---- one-shot solve (one GPU, or opt->n_gpus GPUs of this process) -------- */
int dlp_solve(const dlp_problem* prob, const dlp_options* opt, dlp_result** out);

/* ---- sessions: tableau resident in HBM ---------------------------------- */
/* Single GPU (rank 0 of 1). */
int dlp_session_create(const dlp_problem* prob, const dlp_options* opt, dlp_session** out);
/* Row-block rank of a multi-GPU solve; exchange through RCCL when
 * rccl_unique_id != NULL (128 bytes from dlp_comm_unique_id, identical on every
 * rank), or through caller-driven dlp_session_step_* when it is NULL.  With
 * nranks == 1 and an id, the RCCL exchange path runs on a 1-rank communicator
 * (same results; used to exercise that path on one GPU). */
int dlp_session_create_rank(const dlp_problem* prob, const dlp_options* opt, int rank,
                            int nranks, const void* rccl_unique_id, dlp_session** out);
int dlp_comm_unique_id(void* out128);
/* Launch up to max_pivots more pivots; returns DLP_OK / DLP_UNBOUNDED /
 * DLP_PIVOT_LIMIT / DLP_RUNNING (pivot budget of this call spent). */
int dlp_session_run(dlp_session* s, int64_t max_pivots, int64_t* pivots_done);
/* Caller-driven pivot (external communicator), in this order per pivot:
 *   step_candidate -> all-gather CAND_SEND into CAND_RECV (nranks x 32 B)
 *   step_select    -> all-reduce(MAX, int64) PROW_SEND into PROW_RECV (ld x 8 B)
 *   step_update.   With nranks == 1 no exchange is needed. */
int dlp_session_step_candidate(dlp_session* s);
int dlp_session_step_select(dlp_session* s);
int dlp_session_step_update(dlp_session* s);
int dlp_session_buffer(dlp_session* s, int which, void** dev_ptr, size_t* bytes);
/* Synchronous host copies of an exchange buffer (for host-side communicators). */
int dlp_session_read_buffer(dlp_session* s, int which, void* host, size_t bytes);
int dlp_session_write_buffer(dlp_session* s, int which, const void* host, size_t bytes);
int dlp_session_sync(dlp_session* s);
int dlp_session_status(dlp_session* s, int* status, int64_t* npivots);
int dlp_session_timings(dlp_session* s, double* ms_out /* DLP_NUM_PHASES */, int64_t* nsamples);
/* Update-kernel launches timed (timing >= 1) and their total device time: one
 * rank-1 update per pivot (defer = 1) or one rank-k tableau pass per block. */
int dlp_session_update_stats(dlp_session* s, int64_t* launches, double* ms, int* defer);
int dlp_session_reset_timings(dlp_session* s);
/* Retune the rank-1 update between pivots (results are bit-identical for every
 * setting): variant 0..7 (rows in flight x doubles per lane x colq staging),
 * rows per workgroup band (0 = auto, <= 256), non-temporal loads/stores. */
int dlp_session_set_tuning(dlp_session* s, int update_variant, int rows_per_block, int nontemporal);
int dlp_session_get_tuning(dlp_session* s, int* update_variant, int* rows_per_block, int* nontemporal);
/* 1 when the session solves in the one-launch LDS path (options.small_lp), else 0. */
int dlp_session_small_lp(dlp_session* s, int* small_lp);
/* Lookahead sessions: the CUs the selection chain runs on, the pass on the others (0 = both
 * unmasked).  Auto from the rank's rows; DLP_CHAIN_CUS=n overrides. */
int dlp_session_chain_cus(dlp_session* s, int* cus);
/* Deferred sessions: workgroups per CU allowed for the tableau pass (LDS
 * reservation; 0 = no cap, the default) and its form (-1 = keep):
 *   LDS-staged coefficients: 0 = 2 doubles per lane (K <= 32), 1 / 2 = 1 double
 *   per lane x 2 / 4 rows per iteration;
 *   scalar-load coefficients: 3 = 1 double x 4 rows, 4 = 2 doubles x 2 rows
 *   (K <= 32), 5 = 1 double x 8 rows;
 *   streamed (buffer ops, dense-group ring; K < 16 runs form 3): 6-9 = XCD
 *   band-group order, 10-13 = tile-fastest order, 16-19 = XCD tile-range order,
 *   each as {2 doubles x 2 rows, ring 4 (K <= 32); 2 x 2, ring 2 (K <= 32);
 *   1 x 4, ring 4; 1 x 4, ring 2};
 *   14 = form 4 for full blocks + the streamed partial-block kernel (K <= 32),
 *   15 = the same with the full-block kernel held to 3 waves per SIMD,
 *   20 = form 4 with a 3-deep row prefetch ring (K <= 32),
 *   21 = DPP-broadcast coefficients, 1 double x 2 rows, K = 64 exactly (other K
 *   run form 3),
 *   22 = the same block on the matrix cores (v_mfma_f64_16x16x4f64), K = 64 exactly,
 *   23 = form 21's arithmetic with the rows and coefficients staged through a per-wave
 *   LDS ring by LDS-DMA (4 two-row groups in flight per wave), K = 64 exactly.
 * Default: 21 at K = 64 on a tableau > 1 GiB, 4 at K = 32 there and at K = 16
 * below, else 3.
 * rows_per_block (set_tuning) is the pass's row band (0 = auto: 768 rows at
 * K = 64 on a tableau > 1 GiB, 256 at smaller K there, 64 below).  Results are
 * bit-identical for every setting. */
int dlp_session_set_defer_tuning(dlp_session* s, int occupancy, int form);
/* Deferred single-rank sessions (K <= 32): run the ratio test, the selection
 * and the pivot row as one fused launch per pivot (1) or as two launches (0,
 * the default: the in-launch hand-off costs what the kernel boundary does).
 * Bit-identical either way; timing >= 2 (per-phase events) always uses two
 * launches. */
int dlp_session_set_fused_pivot(dlp_session* s, int on);
/* *on = 1 when the session runs lookahead (dlp_options.lookahead): block b+1 selected
 * while the pass of block b runs on a second tableau buffer.  The step API and pass
 * forms other than 3, 4, 5, 20, 21, 22 and 23 turn it off for the rest of the session. */
int dlp_session_get_lookahead(dlp_session* s, int* on);
/* ---- peer exchange -----------------------------------------------
 * Instead of the RCCL all-gather of the candidates and the int64 MAX all-reduce of the
 * pivot row, the ranks store their candidate into every rank's exchange block and the
 * pivot-row owner stores its row into every rank's block (xGMI peer writes between
 * devices), each message followed by a flag; the waits run inside the select / commit
 * kernels and are bounded.  Results are bit-identical to every other exchange.
 *   one process, any devices (incl. several ranks on ONE device):
 *     dlp_sessions_connect(ranks) once; then dlp_session_run per rank on its own host
 *     thread (distinct devices), or dlp_sessions_run(ranks) from one thread (required
 *     when ranks share a device: it enqueues every rank's sends before any rank's waits);
 *   one process per GPU: dlp_session_exchange_handle (64 B) on every rank, an all-gather
 *     of the handles by the caller, dlp_session_connect_ipc(handles[nranks]); or, with
 *     an RCCL id, dlp_session_set_exchange(s, DLP_XCHG_PEER) does that over RCCL.
 * dlp_session_set_exchange switches between the two on a session that has both (every
 * rank at the same point, between runs). */
#define DLP_XCHG_DEFAULT 0   /* dlp_options.exchange: peer where every rank pair connects, else RCCL */
#define DLP_XCHG_RCCL    1
#define DLP_XCHG_PEER    2
#define DLP_XCHG_HOST    3   /* dlp_session_get_exchange: caller-driven (dlp_session_step_*) */
int dlp_sessions_connect(dlp_session* const* ranks, int nranks);
int dlp_session_exchange_handle(dlp_session* s, void* out64);
int dlp_session_connect_ipc(dlp_session* s, const void* handles /* nranks x 64 B, rank order */);
/* The same connect from records that also carry each rank's device (PCI bus id): ranks that
 * share a device then split the lookahead's chain CUs into disjoint slices (dlp_session_chain_cus;
 * slices under 32 CUs turn the masks off for those ranks), which several rank processes on one
 * GPU need.  dlp_session_exchange_record fills DLP_XREC_BYTES (the exchange
 * block's IPC handle, the bus id); the caller all-gathers them in rank order.  The RCCL-agreed
 * connect (dlp_session_set_exchange / DLP_XCHG_DEFAULT) all-gathers the same records itself.
 * dlp_session_colocated: ranks of the session's exchange on its device (itself included) and its
 * index among them (1, 0 before a connect and after dlp_session_connect_ipc). */
#define DLP_XREC_BYTES 256
int dlp_session_exchange_record(dlp_session* s, void* out /* DLP_XREC_BYTES */);
int dlp_session_connect_records(dlp_session* s, const void* records /* nranks x DLP_XREC_BYTES, rank order */);
int dlp_session_colocated(dlp_session* s, int* n, int* index);
/* The tableau as stored: row stride, RHS column (N, or n when condensed) and whether it is the
 * condensed tableau.  dlp_session_info / _tableau / _read_rows always give the
 * full layout (N + 1 columns, basic columns as unit vectors). */
int dlp_session_storage(dlp_session* s, int64_t* ld, int64_t* ncols, int* condensed);
int dlp_session_set_exchange(dlp_session* s, int mode);
int dlp_session_get_exchange(dlp_session* s, int* mode);
/* Why an auto exchange (DLP_XCHG_DEFAULT) fell back to RCCL ("" when it did not). */
int dlp_session_exchange_reason(dlp_session* s, char* buf, size_t cap);
int dlp_sessions_run(dlp_session* const* ranks, int nranks, int64_t max_pivots, int64_t* pivots_done);

/* Failure containment on the exchange.  A session with an exchange
 * never blocks in a wait that a peer must end: its window waits poll the stream,
 * ncclCommGetAsyncError and an abort word; on an RCCL error, an abort request, a
 * peer-exchange wait that timed out, or a window not complete after `seconds` (the
 * exchange timeout: default 600; 0 = no limit) it raises the device abort word, calls
 * ncclCommAbort and dlp_session_run returns DLP_ERR_RCCL, the status of every exchange
 * failure (the session is then unusable; free it).  A device error returns DLP_ERR_HIP.
 * Each peer-exchange wait on the device is bounded by the same timeout + 5 s.
 * dlp_solve(n_gpus = N) aborts every rank's exchange when one rank fails and returns
 * that rank's error (with the auto exchange, after a failed peer run, the error of the
 * RCCL rerun).  dlp_session_abort may be called from any thread.
 * dlp_session_inject_fault (tests): the (after_polls+1)-th window wait fails as if the
 * exchange had died.
 * Freeing connected ranks: a rank's exchange block receives its peers' stores, so a
 * connected rank session may be freed only after every rank's stream has drained
 * (e.g. a barrier after the last run / result on every rank). */
int dlp_session_set_exchange_timeout(dlp_session* s, double seconds);
int dlp_session_abort(dlp_session* s);
int dlp_session_inject_fault(dlp_session* s, int64_t after_polls);
/* Current deferred-pass settings (K = 1: form -1). */
int dlp_session_get_defer_tuning(dlp_session* s, int* occupancy, int* form, int* K);
int dlp_session_info(dlp_session* s, int64_t* rows_local, int64_t* row_first, int64_t* ld,
                     int64_t* ncols);
/* Copy the local tableau (rows_local+1 rows x ld, objective last) to the host. */
int dlp_session_tableau(dlp_session* s, double* host);
/* Copy local rows [first, first+count) (row rows_local = objective) to the host. */
int dlp_session_read_rows(dlp_session* s, int64_t first, int64_t count, double* host);
int dlp_session_result(dlp_session* s, dlp_result** out);
/* One result for a row-block solve whose rank sessions all live in this
 * process (any order): x covers every basic variable (a single rank's
 * dlp_session_result covers its own rows only). */
int dlp_sessions_result(dlp_session* const* ranks, int nranks, dlp_result** out);
void dlp_session_free(dlp_session* s);

/* ---- batched small LPs ------------------
 * nlp independent LPs of size m x n, LP k generated on the device with seed
 * (seed + k) by the DLP_GEN_* family `kind`; one workgroup per LP solves it
 * with its whole tableau resident in LDS (rule as above, bit-identical to a
 * single-LP solve).  Per-LP outputs (NULL to skip): objective[nlp],
 * status[nlp], npivots[nlp], basis[nlp*m], logs[nlp*log_cap] (first log_cap
 * pivots of each LP).  *kernel_ms gets the solve kernel's device time.
 * Reference analog: the independent per-impression subproblems solved in a
 * loop, R/global_problem.cpp:270-274. */
int dlp_batched_solve(int kind, int64_t nlp, int64_t m, int64_t n, uint64_t seed,
                      const dlp_options* opt, double* objective, int32_t* status,
                      int64_t* npivots, int32_t* basis, dlp_pivot* logs, int64_t log_cap,
                      double* kernel_ms);
/* The batch kernel dlp_batched_solve runs for m x n LPs on `device`: lanes per LP, LPs one CU
 * holds at once (VGPR / LDS occupancy) and whether it is the register-resident kernel (m = 64,
 * n <= 192) or the LDS one.  C5 is bound by per-pivot serial latency x this residency. */
int dlp_batched_occupancy(int64_t m, int64_t n, int device, int32_t* lps_per_cu,
                          int32_t* threads_per_lp, int32_t* register_kernel);

/* ---- multiplicative-weights path ------------------
 * The reference's own epsilon-approximate MW loop (R/allocation_mw.cpp:271-326,
 * sort or binary-search mode) on the GPU for an ad-allocation problem (dlp_problem_create_adalloc),
 * with the fp64 spec of DESIGN.md §9 (fixed tie orders, fixed-order sums,
 * deterministic exp): per impression an upper envelope (wave-level bitonic
 * sort + monotone chain), a global slope sort (hipCUB radix sort), a blocked
 * budget prefix, primal construction, per-advertiser slacks and weights.
 * Scales to the reference's 100k x 1M x 1e-4 scenario, where a dense tableau
 * cannot exist.  Replaces Instance::RunMultiplicativeWeights(T, tol, binary[, scale,
 * intervals]) (R/instance.h:52-55, R/instance.cpp:117-141). */
typedef struct dlp_mw dlp_mw;
typedef struct dlp_mw_options {
    int32_t device;
    int32_t binary;        /* 0 sort mode (R/global_problem.cpp:224-255); 1 threshold search
                              (R/global_problem.cpp:46-222, the mode R/main.cpp:36 runs) with the
                              fp64 stop of DESIGN.md §9 (1e-16 is below fp64 resolution) */
    double  epsilon;       /* default 0.01 (R/main.cpp:33) */
    double  tolerance;     /* numerical_accuracy_tolerance, default 1e-18; tight-set test uses max(tol, 1e-12) */
    double  scale;         /* binary: cr_transition_scale; <= 0 -> 1 - epsilon * 0.001 (R/main.cpp:38) */
    int32_t intervals;     /* binary: critical ratios per level, 1..8, default 3 (R/main.cpp:37) */
    int32_t pad_;
} dlp_mw_options;
typedef struct dlp_mw_iter {   /* per-iteration report (the reference's stdout, R/global_problem.cpp:320,
                                  R/allocation_mw.cpp:214-220,264-268) */
    double  dual_value;
    double  max_infeasibility;
    int32_t infeasible_advertiser;
    int32_t search_levels;     /* binary mode: threshold-search levels this iteration; 0 in sort mode */
    double  min_weight, max_weight, weighted_budget;
} dlp_mw_iter;
void dlp_mw_options_default(dlp_mw_options* opt);
int  dlp_mw_create(const dlp_problem* adalloc, const dlp_mw_options* opt, dlp_mw** out);
/* Run `iterations` more MW iterations; log (may be NULL) gets one entry per iteration;
 * *kernel_ms (may be NULL) the device time of the run. */
int  dlp_mw_run(dlp_mw* mw, int iterations, dlp_mw_iter* log, double* kernel_ms);
/* Averaged and last-iteration primal x in the problem's variable order
 * (dlp_problem_adalloc_bids), and the advertiser weights; NULL pointers skipped. */
int  dlp_mw_solution(dlp_mw* mw, double* x_avg, double* x_current, double* weights);
void dlp_mw_free(dlp_mw* mw);

/* ---- results ------------------------------------------------------------- */
int     dlp_result_status(const dlp_result* r);
double  dlp_result_objective(const dlp_result* r);
int64_t dlp_result_num_pivots(const dlp_result* r);
/* x (n, this rank's basic rows only when nranks > 1), y (m, duals), basis
 * (m_basis).  Dense problems: y_i = z_{n+i}, the max-form dual of row i. */
int dlp_result_x(const dlp_result* r, double* x, int64_t n);
int dlp_result_y(const dlp_result* r, double* y, int64_t m);
int dlp_result_basis(const dlp_result* r, int32_t* basis, int64_t m /* = m_basis */);
/* m_basis: basis length (standard-form rows; m for dense problems);
 * phase1_pivots: pivots of Phase I incl. the artificial drive-out (0 without). */
int dlp_result_info(const dlp_result* r, int64_t* m_basis, int64_t* phase1_pivots);
int dlp_result_pivot_log(const dlp_result* r, dlp_pivot* log, int64_t cap, int64_t* count);
int dlp_result_timings(const dlp_result* r, double* ms_out /* DLP_NUM_PHASES */);
/* dlp_solve(n_gpus >= 1) only: the exchange the result came from (DLP_XCHG_PEER or
 * DLP_XCHG_RCCL; DLP_XCHG_DEFAULT for every other result) and, into reason (cap bytes, NUL
 * terminated), why it is not the peer exchange: the auto exchange could not connect the
 * devices, or the peer run failed and the solve was rerun from the start over RCCL. */
int dlp_result_exchange(const dlp_result* r, int* mode, char* reason, int64_t cap);
void dlp_result_free(dlp_result* r);

#ifdef __cplusplus
}
#endif
#endif /* DLP_H */
