// ref_mw_main.cpp — TEST INFRASTRUCTURE ONLY.  A driver of our own for the
// reference's MW solver, compiled together with the reference's sources where
// they lie (oracle/Makefile target `ref`; binary oracle/_ref/dlp_ref_mw).  The
// reference's main() hard-codes A = I = 1000 and binary mode (R/main.cpp:19-38);
// this driver makes the scenario and the mode (sort / binary) arguments, with
// the rest of the call sequence as R/main.cpp:44-64.
//   usage: dlp_ref_mw A I sparsity iterations sort|binary
#include <cstdlib>
#include <iostream>
#include <string>

#include "instance.h"

int main(int argc, const char* argv[]) {
    using namespace distributed_solver;
    if (argc < 6) {
        std::cerr << "usage: dlp_ref_mw A I sparsity iterations sort|binary\n";
        return 2;
    }
    const int A = std::atoi(argv[1]), I = std::atoi(argv[2]);
    const long double sparsity = (long double)std::atof(argv[3]);   // a double literal, as R/main.cpp:21
    const int iterations = std::atoi(argv[4]);
    const bool binary = std::string(argv[5]) == "binary";
    const long double epsilon = 0.01, tol = 0.000000000000000001;
    Instance inst = Instance(A, I, 1, sparsity, epsilon, 0.25, tol);
    inst.GenerateInstance();
    if (!binary)
        inst.RunMultiplicativeWeights(iterations, tol, false);
    else
        inst.RunMultiplicativeWeights(iterations, tol, true, 1 - epsilon * 0.001, 3);
    std::cout << "finished \n";
    return 0;
}
