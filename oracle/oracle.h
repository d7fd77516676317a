/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement of the pivot rule of
 * SURVEY.md §8(a) (dense-tableau fp64 simplex) and of the instance generators.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as the checker / CPU baseline.  The product
 * (libdlp.so, distributedlpsolver_amd/) never links or calls it.
 *
 * The reference (shidanxu/DistributedLPSolver) has NO simplex:
 * this oracle follows the build-defined rule spec of SURVEY.md §8(a) rows
 * a1-a5/a7, citing the nearest reference analog per function in oracle.cpp.
 * It is pinned by known-answer tests (scipy test_linprog KATs, restated) and
 * by HiGHS objective/x/y fixtures generated in the build container
 * (tests/golden/make_golden.py).  The ad-allocation generator restates
 * R/instance.cpp:32-57 and is pinned against the reference binary built from
 * its own sources (oracle/Makefile target `ref`, outputs in oracle/_ref/).
 *
 * Arithmetic: fp64, explicit std::fma, IEEE division, built with
 * -ffp-contract=off so nothing else is fused.
 */
#ifndef DLP_ORACLE_H
#define DLP_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_pivot {   /* same 32-byte layout as dlp_pivot */
    int32_t q, p, leaving, pad;
    double ratio, objective;
} oracle_pivot;

typedef struct oracle_cand {    /* same 32-byte layout as dlp_candidate */
    double ratio;
    int32_t basis_var, row, valid, pad0;
    double pivot;
} oracle_cand;

typedef struct oracle_opts {
    int32_t pricing;        /* 0 Dantzig->Bland on degeneracy, 1 Bland always */
    double tol_dj, tol_piv;
    int64_t max_pivots;
    int32_t nthreads;       /* OpenMP threads for the update (bit-identical for any value) */
} oracle_opts;

/* Status codes as in dlp.h. */
int oracle_gen_dense(int kind, int64_t m, int64_t n, uint64_t seed, double* A, double* b, double* c);
/* Tableau rows [row_first, row_first+row_count) of the generated LP plus the
 * objective row appended last, leading dimension ld. */
int oracle_gen_tableau(int kind, int64_t m, int64_t n, uint64_t seed, int64_t row_first,
                       int64_t row_count, int64_t ld, double* T, int32_t nthreads);
int64_t oracle_ld(int64_t m, int64_t n);
/* Ad-allocation bids (R/instance.cpp:32-57) via libc srand(1)/rand(); call with
 * NULL arrays to get nnz.  Variables ordered (advertiser asc, impression asc). */
int oracle_gen_adalloc(int A, int I, double sparsity, double scaling, int64_t* nnz,
                       int32_t* adv, int32_t* imp, double* bid, double* budgets,
                       int32_t* draws_per_adv, double* max_bid);

int oracle_solve_dense(int64_t m, int64_t n, const double* A, const double* b, const double* c,
                       const oracle_opts* opt, double* x, double* y, double* obj,
                       int32_t* basis, oracle_pivot* log, int64_t log_cap, int64_t* npivots,
                       int* status);

/* General LP (include/dlp.h "general LPs"; sense 1 = minimise, -1 = maximise):
 * canonical standard form + two-phase simplex with the same rule.  Outputs in
 * user terms; basis (standard-form rows, up to basis_cap); phase1 = pivots of
 * Phase I incl. the drive-out.  Returns -7 when the LP has no constraint rows. */
int oracle_general_std_dims(int64_t m, int64_t n, const double* A, const double* rl,
                            const double* ru, const double* cl, const double* cu, const double* c,
                            double c0, int sense, int64_t* m_std, int64_t* ncols, int64_t* nprice,
                            int64_t* nart);
int oracle_solve_general(int64_t m, int64_t n, const double* A, const double* rl, const double* ru,
                         const double* cl, const double* cu, const double* c, double c0, int sense,
                         const oracle_opts* opt, double tol_feas, double* x, double* y, double* obj,
                         int32_t* basis, int64_t basis_cap, oracle_pivot* log, int64_t log_cap,
                         int64_t* npivots, int64_t* phase1, int* status);

/* Row-slice engine (one simulated rank) for multi-rank protocol tests. */
typedef struct oracle_slice oracle_slice;
int  oracle_slice_create(int64_t m, int64_t n, const double* A, const double* b, const double* c,
                         int64_t row_first, int64_t row_count, const oracle_opts* opt,
                         oracle_slice** out);
/* pricing + local ratio test; returns 0 running, or the terminal status (0 = optimal
 * is reported via *optimal=1). */
int  oracle_slice_candidate(oracle_slice* s, oracle_cand* cand, int* optimal);
/* select the winner among n gathered candidates, record the pivot, and write
 * this rank's all-reduce(MAX) contribution (ld int64): the pivot row's fp64 bits
 * on the owner, INT64_MIN elsewhere.  *unbounded set when no candidate. */
int  oracle_slice_select(oracle_slice* s, const oracle_cand* cands, int n, int64_t* prow_send,
                         int* unbounded);
int  oracle_slice_update(oracle_slice* s, const int64_t* prow_recv);
int64_t oracle_slice_ld(const oracle_slice* s);
int64_t oracle_slice_npivots(const oracle_slice* s);
int  oracle_slice_log(const oracle_slice* s, oracle_pivot* log, int64_t cap);
int  oracle_slice_tableau(const oracle_slice* s, double* T);
void oracle_slice_free(oracle_slice* s);

/* Generate the tableau, run up to k pivots, return the log and copies of the
 * rows listed in rows_idx (row index m = objective row). */
int oracle_run_generated(int kind, int64_t m, int64_t n, uint64_t seed, int64_t k, int32_t nthreads,
                         oracle_pivot* log, int64_t* npivots, const int64_t* rows_idx,
                         int64_t nrows, double* rows_out, int32_t* basis_out);

/* Pivot the generated LP through the ascending stops[0..nstops); at each stop
 * call cb(npivots, T, ld, rows = m+1 (objective row last), log, basis, user). */
typedef void (*oracle_stop_cb)(int64_t npivots, const double* T, int64_t ld, int64_t rows,
                               const oracle_pivot* log, const int32_t* basis, void* user);
int oracle_run_generated_stops(int kind, int64_t m, int64_t n, uint64_t seed, int32_t nthreads,
                               const int64_t* stops, int nstops, oracle_stop_cb cb, void* user);

/* fp64 restatement of the reference's MW loop, sort mode (oracle_mw.cpp): T
 * iterations on the generated ad-allocation instance.  Per-iteration outputs
 * (length T): dual value, max average infeasibility (+ advertiser), min / max
 * weight, weighted budget.  x_avg_out: averaged primal in impression-major
 * order (impression asc, advertiser asc), nnz entries. */
int oracle_mw_run(int A, int I, double sparsity, double scaling, double epsilon, int T, double tol,
                  double* dual, double* infeas, int32_t* infeas_idx, double* wmin, double* wmax,
                  double* budget_w, double* x_avg_out, double* weights_out, int64_t* nnz_out);
/* The same, either mode: binary = 1 selects the threshold search of
 * R/global_problem.cpp:46-222 (spec in oracle_mw.cpp's header) with
 * cr_transition_scale `scale` and `intervals` critical ratios per level (1..8).
 * levels_out (T entries) gets the number of search levels per iteration,
 * interval_out (2T) the final (lower, upper) (cr, cr for an exact hit); both
 * may be NULL and are untouched in sort mode. */
int oracle_mw_run_mode(int A, int I, double sparsity, double scaling, double epsilon, int T,
                       double tol, int binary, double scale, int intervals, double* dual,
                       double* infeas, int32_t* infeas_idx, double* wmin, double* wmax,
                       double* budget_w, double* x_avg_out, double* weights_out, int64_t* nnz_out,
                       int32_t* levels_out, double* interval_out);
double oracle_sum_blocked(const double* x, int64_t n);
double oracle_dexp(double x);
double oracle_sum_fixed(const double* x, int64_t n);

/* CPU baseline: generate the tableau, do `warmup` pivots, time `k` pivots. */
int oracle_bench_pivots(int kind, int64_t m, int64_t n, uint64_t seed, int64_t warmup, int64_t k,
                        int32_t nthreads, double* seconds, int64_t* done, double* gen_seconds);
/* CPU baseline over several thread counts on ONE generated LP: one warm-up
 * pivot, then nrun consecutive windows (threads[r] threads, at most max_k[r]
 * pivots or budget_s[r] seconds); secs[r], done[r] per window. */
int oracle_bench_windows(int kind, int64_t m, int64_t n, uint64_t seed, int32_t gen_threads,
                         int nrun, const int32_t* threads, const int64_t* max_k,
                         const double* budget_s, double* secs, int64_t* done,
                         double* gen_seconds);

#ifdef __cplusplus
}
#endif
#endif
