// dlp_host.h — host-side objects behind the C ABI (not public).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "dlp.h"

namespace dlp {

enum ProblemKind { PROB_DENSE = 0, PROB_RANDOM = 1, PROB_ADALLOC = 2, PROB_GENERAL = 3 };

struct AdAlloc {
    int num_advertisers = 0, num_impressions = 0;
    std::vector<int32_t> adv, imp;   // variable k = (adv[k], imp[k]), ordered (a, i) ascending
    std::vector<double> bid, budget;
    std::vector<int32_t> draws;      // draws per advertiser (loop bound check, R/instance.cpp:44)
    double max_bid = 0.0;
    double sparsity = 0.0;           // bid_sparsity as given (MW width, R/allocation_mw.cpp:155)
};

int build_adalloc(int A, int I, double sparsity, double scaling, AdAlloc* out);

// User-level general LP (dlp_problem_create_general / _mps).
struct General {
    int64_t m = 0, n = 0;
    std::vector<double> A;                       // m x n row-major
    std::vector<double> row_lo, row_hi, col_lo, col_hi, c;
    double c0 = 0.0;
    int sense = DLP_MINIMIZE;
};

enum RowType : int8_t { ROW_L = 0, ROW_G = 1, ROW_E = 2 };
enum VarKind : int8_t { VAR_LO = 0, VAR_HI = 1, VAR_FREE = 2 };

// Canonical standard form of a General (spec: include/dlp.h, "general LPs").
struct StdForm {
    int64_t m = 0;           // constraint rows
    int64_t ns = 0;          // structural columns
    int64_t nslack = 0;      // slack / surplus columns (one per L / G row)
    int64_t nart = 0;        // artificial columns (one per G / E row)
    std::vector<double> A;   // m x ns row-major
    std::vector<double> b;   // m, >= 0
    std::vector<int8_t> type;
    std::vector<int32_t> slack_col, art_col;   // per row: absolute column, -1 when none
    std::vector<double> c;   // ns, max form
    // back-mapping to user variables / rows
    std::vector<int32_t> var_col;   // first structural column of user variable j
    std::vector<int8_t> var_kind;
    std::vector<double> var_const;  // lo (VAR_LO) or hi (VAR_HI)
    std::vector<int32_t> user_row;  // per std row: user row (-1 for bound rows)
    std::vector<double> row_sign;   // per std row: +1 / -1 (negated)
    double obj_sign = 1.0;          // user objective = obj_sign * z_N + obj_const
    double obj_const = 0.0;         // c0 + fma-chain over j ascending of c_j * const_j
    int64_t ncols() const { return ns + nslack + nart; }
    int64_t nprice() const { return ns + nslack; }
};

int build_stdform(const General& g, StdForm* out);
int parse_mps(const char* path, General* out);

void set_error(const std::string& msg);

}  // namespace dlp

struct dlp_problem {
    int kind = dlp::PROB_DENSE;
    int64_t m = 0, n = 0;
    std::vector<double> A, b, c;   // PROB_DENSE
    int gen_kind = 0;              // PROB_RANDOM
    uint64_t seed = 0;
    dlp::AdAlloc ad;               // PROB_ADALLOC
    dlp::General gen;              // PROB_GENERAL
    dlp::StdForm sf;               // PROB_GENERAL
};

struct dlp_result {
    int status = DLP_ERR_STATE;
    double objective = 0.0;
    int64_t npivots = 0;
    int64_t phase1_pivots = 0;
    int64_t m = 0, n = 0;
    std::vector<double> x, y;
    std::vector<int32_t> basis;
    std::vector<dlp_pivot> log;
    double timings[DLP_NUM_PHASES] = {0, 0, 0, 0};
    int exchange = DLP_XCHG_DEFAULT;   // dlp_solve(n_gpus): the exchange the result came from
    std::string exchange_reason;       // why not the peer exchange ("" when it was, or not a solve)
};
