// The reference's driver call sequence (R/main.cpp:44-64), compiled against the
// drop-in facade (include/distributed_solver/instance.h) instead of the
// reference sources.  argv: A I sparsity [solve|simplex] [iterations] [sort]
//   no mode: GenerateInstance only (host-only, prints the topology);
//   "solve": R/main.cpp:58-64 literally (use_binary_search = true: the
//            threshold-search MW loop on the GPU; a trailing "sort" flips the
//            flag as R/main.cpp:36's comment describes) -> per-iteration
//            "Dual Value = ..." lines;
//   "simplex": the added exact entry RunSimplex (dense-tableau simplex).
// Both solve modes end with one "status ... pivots ... objective ..." line.
#include <cstdlib>
#include <iostream>
#include <string>

#include "distributed_solver/instance.h"

int main(int argc, const char* argv[]) {
    using namespace distributed_solver;
    int A = argc > 1 ? std::atoi(argv[1]) : 1000;
    int I = argc > 2 ? std::atoi(argv[2]) : 1000;
    long double sparsity = argc > 3 ? (long double)std::atof(argv[3]) : 0.1;
    const std::string mode = argc > 4 ? argv[4] : "";
    int num_iterations = argc > 5 ? std::atoi(argv[5]) : 300;
    long double epsilon = 0.01;
    long double numerical_accuracy_tolerance = 0.000000000000000001;
    bool use_binary_search = true;	// Setting this to false runs the sort method
    if (argc > 6 && std::string(argv[6]) == "sort") use_binary_search = false;
    int num_bin_intervals = 3;
    long double cr_transition_scale = 1 - epsilon * 0.001;

    Instance inst = Instance(A, I, 1, sparsity, epsilon, 0.25, numerical_accuracy_tolerance);
    inst.GenerateInstance();
    if (mode == "solve") {
        if (!use_binary_search) {
            inst.RunMultiplicativeWeights(num_iterations, numerical_accuracy_tolerance, use_binary_search);
        } else {
            inst.RunMultiplicativeWeights(num_iterations, numerical_accuracy_tolerance, use_binary_search,
                                          cr_transition_scale, num_bin_intervals);
        }
    } else if (mode == "simplex") {
        dlp_options o;
        dlp_options_default(&o);
        inst.RunSimplex(o);
    }
    if (!mode.empty()) {
        std::cout.precision(17);
        std::cout << "status " << inst.Status() << " pivots " << inst.NumPivots() << " objective "
                  << (double)inst.DualValue() << " revenue " << (double)inst.Revenue()
                  << " max_infeasibility " << (double)inst.MaxInfeasibility() << "\n";
    }
    std::cout << "finished \n";
    return 0;
}
