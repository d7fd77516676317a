// instance.h — C++ facade with the reference's problem-loading / solver-entry
// / result surface, over the C ABI of include/dlp.h.
//
// Same constructor, GenerateInstance and RunMultiplicativeWeights signatures
// as R/instance.h:41-53 (R/ = /root/reference/DistributedLPSolver/
// DistributedLPSolver/), so the reference's caller R/main.cpp compiles and
// links unchanged against it (tests/test_facade.py::test_reference_main_compiles).
// As R/instance.h:11-18 does, it gives its includers <ext/hash_map>,
// <fstream>, <iostream>, <string>, <vector> and `using namespace std;`
// (R/main.cpp:71 writes `cout` and `endl` unqualified).  What changes underneath: RunMultiplicativeWeights runs
// the reference's epsilon-approximate MW loop on the GPU (dlp_mw_*), and the
// added RunSimplex solves the same LP EXACTLY with the MI355X dense-tableau
// simplex.  The result the reference keeps private (solution_, R/instance.h:34)
// and prints ("Dual Value", R/global_problem.cpp:320-322) is available through
// Solution() / DualValue() / MWLog().
#pragma once

// <ext/hash_map> is libstdc++'s pre-C++11 hash table, the reference's
// container (R/instance.h:11); silence its "deprecated header" warning here
#ifndef _GLIBCXX_PERMIT_BACKWARD_HASH
#define _GLIBCXX_PERMIT_BACKWARD_HASH
#endif
#include <ext/hash_map>
#include <fstream>
#include <iostream>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../dlp.h"

using namespace std;   // R/instance.h:18: the reference's includers rely on it

namespace distributed_solver {

// One advertiser's primal entries: impression -> (current x, running-average x),
// the element type of the reference's solution_ and of its statics'
// parameters (R/instance.h:34,55,57): the same __gnu_cxx::hash_map.
typedef __gnu_cxx::hash_map<int, std::pair<long double, long double> > PrimalRow;

class Instance {
  public:
    // R/instance.h:41-42.  num_slots must be 1 (every reference scenario).
    Instance(int num_advertisers, int num_impressions, int num_slots, long double bid_sparsity,
             long double epsilon, long double scaling_factor,
             long double numerical_accuracy_tolerance);
    ~Instance();
    Instance(const Instance&) = delete;
    Instance& operator=(const Instance&) = delete;
    Instance(Instance&& o) noexcept;

    // R/instance.h:46: srand(1) bid generation (R/instance.cpp:32-57), printed
    // topology as the reference prints it (R/instance.cpp:178-185).
    void GenerateInstance();
    // R/instance.cpp:136-141 (called by the constructor, as in the reference).
    void SetBudgets();
    // R/instance.h:47-48.  The reference's bodies have every file operation
    // commented out (R/instance.cpp:59-115); these write what those comments
    // describe: <handle>AxIxSxSPARSITY.csv, one line per advertiser of
    // "impression,bid," pairs (impressions ascending, std::to_string formatting).
    // GenerateAndWriteInstance draws the bids as GenerateInstance does and
    // writes the one shard <name>.csv@0 (the reference's shard count is an
    // uninitialised member, R/instance.h:26).  Both return nothing and print as
    // the reference prints; a file that cannot be opened throws.
    void WriteInstanceToCSV(std::string file_name_handle);
    void GenerateAndWriteInstance(std::string file_name_handle);

    // R/instance.h:52-53.  The reference's MW loop on the GPU (dlp_mw_*, fp64
    // spec of DESIGN.md §9): binary = false sort mode, binary = true the
    // threshold search with cr_transition_scale `scale` and `intervals`
    // critical ratios per level (3-argument form: 1 - epsilon * 0.001 and 3,
    // R/main.cpp:37-38); prints the reference's per-iteration "Dual Value" /
    // infeasibility / weight lines.
    void RunMultiplicativeWeights(long double num_iterations,
                                  long double numerical_accuracy_tolerance, bool binary);
    void RunMultiplicativeWeights(long double num_iterations,
                                  long double numerical_accuracy_tolerance, bool binary,
                                  long double scale, int intervals);

    // R/instance.h:55-57 (statics over a caller's solution vector, as the MW
    // loop uses them, R/allocation_mw.cpp:287-291; and BuildPrimals, public in
    // the reference): running average x_avg = (t-1)/t x_avg + 1/t x
    // (R/instance.cpp:143-152); one (0, 0) pair per bid (R/instance.cpp:154-165);
    // current x := 0 (R/instance.cpp:167-176).
    static void UpdateAvgPrimal(int t, std::vector<PrimalRow>* solution);
    void BuildPrimals();
    static void ResetCurrentPrimal(std::vector<PrimalRow>* sol);

    // Added entry: solve the same LP EXACTLY with the dense-tableau simplex;
    // returns a dlp status; Solution() pairs are then (x*, x*).
    int RunSimplex(const dlp_options& options);
    const std::vector<dlp_mw_iter>& MWLog() const { return mw_log_; }

    // Results.  Solution()[a][i] = (current x_ai, averaged x_ai) as in the
    // reference's solution_ (both equal the exact optimum here).
    const std::vector<PrimalRow>& Solution() const { return solution_; }
    long double DualValue() const { return dual_value_; }
    long double MaxInfeasibility() const;   // max_a (sum_i b_ai x_ai - B_a)/B_a, cf. R/allocation_mw.cpp:205-232
    long double Revenue() const;            // sum b_ai x_ai, cf. R/allocation_mw.cpp:235-251
    int64_t NumPivots() const { return num_pivots_; }
    int Status() const { return status_; }
    const std::vector<long double>& Budgets() const { return budgets_; }
    const std::vector<std::unordered_map<int, long double>>& Bids() const { return bids_matrix_; }

    long double max_bid_ = 0;   // public in the reference (R/instance.h:43)
    bool verbose = true;        // print as the reference does

  private:
    void ReportGraphTopology();
    std::string CsvName(const std::string& handle) const;

    int num_advertisers_, num_impressions_, num_slots_;
    long double bid_sparsity_, epsilon_, scaling_factor_, numerical_accuracy_tolerance_;
    std::vector<long double> budgets_;
    std::vector<std::unordered_map<int, long double>> bids_matrix_;
    std::vector<std::unordered_map<int, long double>> transpose_bids_matrix_;
    std::vector<PrimalRow> solution_;
    dlp_problem* problem_ = nullptr;
    long double dual_value_ = 0;
    std::vector<dlp_mw_iter> mw_log_;
    int64_t num_pivots_ = 0;
    int status_ = DLP_ERR_STATE;
};

}  // namespace distributed_solver
