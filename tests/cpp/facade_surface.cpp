// The rest of the reference's public Instance surface (R/instance.h:41-57),
// host-only: WriteInstanceToCSV, GenerateAndWriteInstance, the static
// UpdateAvgPrimal / ResetCurrentPrimal and the public BuildPrimals, called as
// the reference's code calls them (R/allocation_mw.cpp:287-291).
// argv: A I sparsity out_handle.  Prints one "check ..." line per property.
#include <cmath>
#include <cstdlib>
#include <iostream>
#include <string>
#include <vector>

#include "distributed_solver/instance.h"

int main(int argc, const char* argv[]) {
    using namespace distributed_solver;
    const int A = std::atoi(argv[1]), I = std::atoi(argv[2]);
    const long double sparsity = (long double)std::atof(argv[3]);
    const std::string handle = argv[4];
    Instance inst(A, I, 1, sparsity, 0.01, 0.25, 1e-18L);
    inst.verbose = false;
    inst.GenerateAndWriteInstance(handle);
    inst.WriteInstanceToCSV(handle);
    inst.BuildPrimals();
    std::vector<PrimalRow> sol = inst.Solution();
    size_t pairs = 0;
    for (auto& row : sol)
        for (auto& kv : row) {
            kv.second.first = 1.0L;   // current x = 1 for every bid
            ++pairs;
        }
    for (int t = 1; t <= 4; ++t) Instance::UpdateAvgPrimal(t, &sol);   // average of 1s = 1
    bool avg_ok = true;
    for (auto& row : sol)
        for (auto& kv : row) avg_ok = avg_ok && kv.second.second == 1.0L;
    Instance::ResetCurrentPrimal(&sol);
    bool reset_ok = true;
    for (auto& row : sol)
        for (auto& kv : row) reset_ok = reset_ok && kv.second.first == 0.0L && kv.second.second == 1.0L;
    std::cout << "check pairs " << pairs << "\n";
    std::cout << "check avg " << avg_ok << " reset " << reset_ok << "\n";
    return avg_ok && reset_ok ? 0 : 1;
}
