// dlp_host.h — host-side objects behind the C ABI (not public).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "dlp.h"

namespace dlp {

enum ProblemKind { PROB_DENSE = 0, PROB_RANDOM = 1, PROB_ADALLOC = 2 };

struct AdAlloc {
    int num_advertisers = 0, num_impressions = 0;
    std::vector<int32_t> adv, imp;   // variable k = (adv[k], imp[k]), ordered (a, i) ascending
    std::vector<double> bid, budget;
    std::vector<int32_t> draws;      // draws per advertiser (loop bound check, R/instance.cpp:44)
    double max_bid = 0.0;
    double sparsity = 0.0;           // bid_sparsity as given (MW width, R/allocation_mw.cpp:155)
};

int build_adalloc(int A, int I, double sparsity, double scaling, AdAlloc* out);

void set_error(const std::string& msg);

}  // namespace dlp

struct dlp_problem {
    int kind = dlp::PROB_DENSE;
    int64_t m = 0, n = 0;
    std::vector<double> A, b, c;   // PROB_DENSE
    int gen_kind = 0;              // PROB_RANDOM
    uint64_t seed = 0;
    dlp::AdAlloc ad;               // PROB_ADALLOC
};

struct dlp_result {
    int status = DLP_ERR_STATE;
    double objective = 0.0;
    int64_t npivots = 0;
    int64_t m = 0, n = 0;
    std::vector<double> x, y;
    std::vector<int32_t> basis;
    std::vector<dlp_pivot> log;
    double timings[DLP_NUM_PHASES] = {0, 0, 0, 0};
};
