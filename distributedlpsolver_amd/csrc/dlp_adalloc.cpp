// dlp_adalloc.cpp — the reference's ad-allocation instance, regenerated
// bit-exactly, with glibc's TYPE_3 additive-feedback
// rand() embedded so the library keeps no hidden global RNG state.
//
// Restates Instance::GenerateInstance (R/instance.cpp:32-57) and
// Instance::SetBudgets (R/instance.cpp:136-141):
//   srand(1); for each advertiser a: draw while i < (long double)sparsity * I:
//       index = rand() % I;  bid = (long double)(rand()+1) / RAND_MAX;
//       bids[a][index] = bid   (hash_map assignment: a repeated draw overwrites)
//   B_a = 0.5L * (I / A) * scaling   (integer I / A)
// The LP built from it (R/allocation_mw.cpp:163-171 slacks, :129-138 subproblem):
//   max sum b_ai x_ai  s.t.  sum_i b_ai x_ai <= B_a,  sum_a x_ai <= 1,  x >= 0.
#include <cstdint>
#include <map>
#include <vector>

#include "dlp_host.h"

namespace dlp {

namespace {
// glibc random_r TYPE_3 (degree 31, separation 3), seeded as srand(seed).
class GlibcRand {
  public:
    explicit GlibcRand(uint32_t seed) {
        int32_t r[34];
        r[0] = (int32_t)(seed == 0 ? 1 : seed);
        for (int i = 1; i < 31; ++i) {
            // r[i] = (16807 * r[i-1]) % 2147483647 via Schrage, as glibc does.
            const int32_t hi = r[i - 1] / 127773, lo = r[i - 1] % 127773;
            int32_t word = 16807 * lo - 2836 * hi;
            if (word < 0) word += 2147483647;
            r[i] = word;
        }
        for (int i = 0; i < 31; ++i) state_[i] = (uint32_t)r[i];
        f_ = 3;   // fptr = &state[SEP]
        b_ = 0;   // rptr = &state[0]
        for (int i = 0; i < 310; ++i) next();   // glibc discards 10 * degree outputs
    }
    int32_t next() {
        state_[f_] += state_[b_];
        const int32_t result = (int32_t)(state_[f_] >> 1);
        f_ = (f_ + 1) % 31;
        b_ = (b_ + 1) % 31;
        return result;
    }

  private:
    uint32_t state_[31];
    int f_, b_;
};
constexpr int32_t kRandMax = 2147483647;
}  // namespace

int build_adalloc(int A, int I, double sparsity, double scaling, AdAlloc* out) {
    if (A <= 0 || I <= 0 || !(sparsity >= 0.0)) return DLP_ERR_ARG;
    GlibcRand rng(1);
    std::vector<std::map<int, double>> rows(A);
    const long double bound = (long double)sparsity * (long double)I;
    long double max_bid = 0;
    out->draws.assign(A, 0);
    for (int a = 0; a < A; ++a) {
        for (int i = 0; i < bound; ++i) {
            const int index = rng.next() % I;
            const long double bid = (long double)(rng.next() + 1) / (long double)kRandMax;
            if (max_bid < bid) max_bid = bid;
            rows[a][index] = (double)bid;
            ++out->draws[a];
        }
    }
    out->num_advertisers = A;
    out->num_impressions = I;
    out->adv.clear();
    out->imp.clear();
    out->bid.clear();
    for (int a = 0; a < A; ++a)
        for (const auto& kv : rows[a]) {
            out->adv.push_back(a);
            out->imp.push_back(kv.first);
            out->bid.push_back(kv.second);
        }
    out->budget.assign(A, (double)(0.5L * (long double)(I / A) * (long double)scaling));
    out->max_bid = (double)max_bid;
    out->sparsity = sparsity;
    return DLP_OK;
}

}  // namespace dlp
