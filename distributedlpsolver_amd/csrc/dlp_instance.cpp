// dlp_instance.cpp — the reference-signature facade (include/distributed_solver/
// instance.h) over the C ABI.  Reference: R/instance.{h,cpp}.
#include "distributed_solver/instance.h"

#include <algorithm>
#include <fstream>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

namespace distributed_solver {

Instance::Instance(int num_advertisers, int num_impressions, int num_slots,
                   long double bid_sparsity, long double epsilon, long double scaling_factor,
                   long double numerical_accuracy_tolerance)
    : num_advertisers_(num_advertisers),
      num_impressions_(num_impressions),
      num_slots_(num_slots),
      bid_sparsity_(bid_sparsity),
      epsilon_(epsilon),
      scaling_factor_(scaling_factor),
      numerical_accuracy_tolerance_(numerical_accuracy_tolerance) {
    budgets_.assign(num_advertisers_ > 0 ? num_advertisers_ : 0, 0.0L);
    SetBudgets();
}

Instance::~Instance() {
    if (problem_) dlp_problem_free(problem_);
}

Instance::Instance(Instance&& o) noexcept
    : max_bid_(o.max_bid_),
      verbose(o.verbose),
      num_advertisers_(o.num_advertisers_),
      num_impressions_(o.num_impressions_),
      num_slots_(o.num_slots_),
      bid_sparsity_(o.bid_sparsity_),
      epsilon_(o.epsilon_),
      scaling_factor_(o.scaling_factor_),
      numerical_accuracy_tolerance_(o.numerical_accuracy_tolerance_),
      budgets_(std::move(o.budgets_)),
      bids_matrix_(std::move(o.bids_matrix_)),
      transpose_bids_matrix_(std::move(o.transpose_bids_matrix_)),
      solution_(std::move(o.solution_)),
      problem_(o.problem_),
      dual_value_(o.dual_value_),
      num_pivots_(o.num_pivots_),
      status_(o.status_) {
    o.problem_ = nullptr;
}

// R/instance.cpp:136-141 (average bid 0.5, integer I/A, scaling factor).
void Instance::SetBudgets() {
    const long double average_bid = 0.5;
    for (int a = 0; a < num_advertisers_; ++a)
        budgets_[a] = average_bid * (num_impressions_ / num_advertisers_) * scaling_factor_;
}

// R/instance.cpp:32-57; the bids come from libdlp's bit-exact restatement.
void Instance::GenerateInstance() {
    if (problem_) dlp_problem_free(problem_);
    problem_ = nullptr;
    int rc = dlp_problem_create_adalloc(num_advertisers_, num_impressions_, num_slots_,
                                        (double)bid_sparsity_, (double)scaling_factor_, &problem_);
    if (rc != DLP_OK) throw std::runtime_error(std::string("GenerateInstance: ") + dlp_last_error());
    int64_t nnz = 0;
    dlp_problem_adalloc_bids(problem_, &nnz, nullptr, nullptr, nullptr);
    std::vector<int32_t> adv(nnz), imp(nnz);
    std::vector<double> bid(nnz);
    dlp_problem_adalloc_bids(problem_, &nnz, adv.data(), imp.data(), bid.data());
    bids_matrix_.assign(num_advertisers_, {});
    transpose_bids_matrix_.assign(num_impressions_, {});
    max_bid_ = 0;
    for (int64_t k = 0; k < nnz; ++k) {
        bids_matrix_[adv[k]][imp[k]] = bid[k];
        transpose_bids_matrix_[imp[k]][adv[k]] = bid[k];
        max_bid_ = std::max<long double>(max_bid_, bid[k]);
    }
    if (verbose) {
        std::cout << "Generated instance \n";
        ReportGraphTopology();
    }
}

// R/instance.cpp:178-185.
void Instance::ReportGraphTopology() {
    for (int a = 0; a < (int)bids_matrix_.size(); ++a)
        std::cout << "Advertiser " << a << " degree is " << bids_matrix_[a].size() << "\n";
    for (int i = 0; i < (int)transpose_bids_matrix_.size(); ++i)
        std::cout << "Impression " << i << " degree is " << transpose_bids_matrix_[i].size() << "\n";
}

// R/instance.cpp:154-165: one (current, average) pair per bid.
void Instance::BuildPrimals() {
    solution_.assign(num_advertisers_, {});
    for (int a = 0; a < num_advertisers_ && a < (int)bids_matrix_.size(); ++a)
        for (const auto& kv : bids_matrix_[a]) solution_[a][kv.first] = {0.0L, 0.0L};
}

// R/instance.cpp:143-152, in long double as there.
void Instance::UpdateAvgPrimal(int t, std::vector<PrimalRow>* solution) {
    for (auto& row : *solution)
        for (auto& kv : row)
            kv.second.second = (long double)(t - 1) / t * kv.second.second +
                               (long double)1 / t * kv.second.first;
}

// R/instance.cpp:167-176.
void Instance::ResetCurrentPrimal(std::vector<PrimalRow>* sol) {
    for (auto& row : *sol)
        for (auto& kv : row) kv.second.first = 0.0;
}

// The file name of the reference's commented-out writer (R/instance.cpp:63).
std::string Instance::CsvName(const std::string& handle) const {
    return handle + std::to_string(num_advertisers_) + "x" + std::to_string(num_impressions_) + "x" +
           std::to_string(num_slots_) + "x" + std::to_string(bid_sparsity_) + ".csv";
}

static void write_bid_rows(std::ofstream& file,
                           const std::vector<std::unordered_map<int, long double>>& bids) {
    for (const auto& adv : bids) {
        std::vector<std::pair<int, long double>> row(adv.begin(), adv.end());
        std::sort(row.begin(), row.end());
        std::string line;
        for (const auto& kv : row) line += std::to_string(kv.first) + "," + std::to_string(kv.second) + ",";
        file << line << "\n";
    }
}

// R/instance.cpp:59-86 (its file operations are comments there; done here).
void Instance::WriteInstanceToCSV(std::string file_name_handle) {
    const std::string name = CsvName(file_name_handle);
    if (verbose) std::cout << file_name_handle + "\n" << "Writing instance " + name + "\n";
    std::ofstream file(name);
    if (!file) throw std::runtime_error("WriteInstanceToCSV: cannot open " + name);
    write_bid_rows(file, bids_matrix_);
}

// R/instance.cpp:88-115: srand(1) bids, written as one shard.
void Instance::GenerateAndWriteInstance(std::string file_name_handle) {
    const bool v = verbose;
    verbose = false;
    GenerateInstance();
    verbose = v;
    const std::string name = CsvName(file_name_handle) + "@0";
    if (verbose) std::cout << "Writing instance " + name + "\n";
    std::ofstream file(name);
    if (!file) throw std::runtime_error("GenerateAndWriteInstance: cannot open " + name);
    write_bid_rows(file, bids_matrix_);
}

int Instance::RunSimplex(const dlp_options& options) {
    if (!problem_) GenerateInstance();
    BuildPrimals();
    dlp_result* r = nullptr;
    status_ = dlp_solve(problem_, &options, &r);
    if (status_ < 0) return status_;
    status_ = dlp_result_status(r);
    int64_t m = 0, n = 0;
    dlp_problem_dims(problem_, &m, &n);
    std::vector<double> x(n);
    dlp_result_x(r, x.data(), n);
    dual_value_ = dlp_result_objective(r);
    num_pivots_ = dlp_result_num_pivots(r);
    dlp_result_free(r);
    std::vector<int32_t> adv(n), imp(n);
    int64_t nnz = n;
    dlp_problem_adalloc_bids(problem_, &nnz, adv.data(), imp.data(), nullptr);
    for (int64_t k = 0; k < n; ++k) solution_[adv[k]][imp[k]] = {x[k], x[k]};
    return status_;
}

// R/instance.cpp:117-141 -> R/allocation_mw.cpp:271-326: the MW loop on the
// GPU (dlp_mw_*), sort mode (binary = false) or the threshold search
// (binary = true, R/global_problem.cpp:46-222, the mode R/main.cpp:36 runs)
// with the fp64 spec of DESIGN.md §9.  Prints the reference's per-iteration
// report lines.
namespace {
void run_mw(dlp_problem* problem, long double epsilon, int T, long double tol, bool binary,
            double scale, int intervals, std::vector<dlp_mw_iter>& log, std::vector<double>& xa,
            std::vector<double>& xc) {
    dlp_mw_options o;
    dlp_mw_options_default(&o);
    o.epsilon = (double)epsilon;
    o.tolerance = (double)tol;
    o.binary = binary ? 1 : 0;
    o.scale = scale;
    o.intervals = intervals;
    dlp_mw* mw = nullptr;
    int rc = dlp_mw_create(problem, &o, &mw);
    if (rc != DLP_OK) throw std::runtime_error(std::string("RunMultiplicativeWeights: ") + dlp_last_error());
    log.assign(T > 0 ? T : 1, dlp_mw_iter{});
    rc = dlp_mw_run(mw, T, log.data(), nullptr);
    if (rc != DLP_OK) {
        dlp_mw_free(mw);
        throw std::runtime_error(std::string("RunMultiplicativeWeights: ") + dlp_last_error());
    }
    int64_t m = 0, n = 0;
    dlp_problem_dims(problem, &m, &n);
    xa.assign(n, 0.0);
    xc.assign(n, 0.0);
    dlp_mw_solution(mw, xa.data(), xc.data(), nullptr);
    dlp_mw_free(mw);
}
}  // namespace

void Instance::RunMultiplicativeWeights(long double num_iterations,
                                        long double numerical_accuracy_tolerance, bool binary) {
    // The reference's 3-argument path leaves cr_transition_scale_ and
    // num_bin_intervals_ unset (R/global_problem.cpp:18-27); binary = true here
    // takes R/main.cpp's values (1 - epsilon * 0.001, 3).
    RunMultiplicativeWeights(num_iterations, numerical_accuracy_tolerance, binary,
                             1 - epsilon_ * 0.001, 3);
}

void Instance::RunMultiplicativeWeights(long double num_iterations,
                                        long double numerical_accuracy_tolerance, bool binary,
                                        long double scale, int intervals) {
    if (!problem_) GenerateInstance();
    BuildPrimals();
    const int T = (int)num_iterations;
    std::vector<dlp_mw_iter> log;
    std::vector<double> xa, xc;
    run_mw(problem_, epsilon_, T, numerical_accuracy_tolerance, binary, (double)scale, intervals, log,
           xa, xc);
    const int64_t n = (int64_t)xa.size();
    std::vector<int32_t> adv(n), imp(n);
    int64_t nnz = n;
    dlp_problem_adalloc_bids(problem_, &nnz, adv.data(), imp.data(), nullptr);
    for (int64_t k = 0; k < n; ++k) solution_[adv[k]][imp[k]] = {xc[k], xa[k]};
    mw_log_.assign(log.begin(), log.begin() + (T > 0 ? T : 0));
    for (int t = 0; t < T && verbose; ++t) {
        std::cout << "Entering iteration " << t + 1 << "\n";
        std::cout << "Dual Value = " << log[t].dual_value << "\n";
        std::cout << "At iteration " << t + 1 << ", max infeasiblity was " << log[t].max_infeasibility
                  << " on constraint " << log[t].infeasible_advertiser << "\n";
        std::cout << "min weight = " << log[t].min_weight << ", max weight = " << log[t].max_weight
                  << "\n";
    }
    dual_value_ = T > 0 ? log[T - 1].dual_value : 0.0L;
    status_ = DLP_OK;
    num_pivots_ = 0;
}

long double Instance::MaxInfeasibility() const {
    long double worst = 0;
    for (int a = 0; a < num_advertisers_ && a < (int)solution_.size(); ++a) {
        long double spend = 0;
        for (const auto& kv : solution_[a]) spend += kv.second.first * bids_matrix_[a].at(kv.first);
        worst = std::max(worst, (spend - budgets_[a]) / budgets_[a]);
    }
    return worst;
}

long double Instance::Revenue() const {
    long double rev = 0;
    for (int a = 0; a < (int)solution_.size(); ++a)
        for (const auto& kv : solution_[a]) rev += kv.second.first * bids_matrix_[a].at(kv.first);
    return rev;
}

}  // namespace distributed_solver
