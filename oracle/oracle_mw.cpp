// oracle_mw.cpp — TEST INFRASTRUCTURE ONLY.  fp64 restatement of the
// reference's multiplicative-weights (MW) iteration in SORT and BINARY
// (threshold-search) mode, the CPU checker of the GPU
// MW path.
//
// The reference computes in x87 long double and leaves several choices to
// std::sort / hash_map order; this restatement fixes every such choice (the
// "MW fp64 spec") so that a GPU implementation can be compared
// bit for bit:
//   * bids of impression i in advertiser-ascending order; hull sort key
//     (coefficient desc, price desc, advertiser asc)        R/upper_envelope.h:27-32
//   * monotone chain, pop while cross <= 1e-14, cross = d1 - d2 (no fma)
//                                                           R/upper_envelope.cpp:15-38
//   * envelope points / budget cutoffs as R/subproblem.cpp:210-231
//   * global regions sorted by (slope desc, impression asc, region asc)
//                                                           R/global_problem.cpp:224-255
//   * remaining budget = B - S_k, S_k the exclusive prefix of region widths in
//     sorted order computed in chunks of 256 (sequential inside a chunk, chunk
//     offsets sequential); increment = min(max(B - S_k, 0), width)
//   * dual value and weighted budget: sum_fixed (64 strided sequential chains,
//     then the halving tree s_l += s_{l+w}, w = 32..1)
//   * primal construction as R/global_problem.cpp:325-412 with the tight-set
//     tolerance max(numerical_accuracy_tolerance, 1e-12) (1e-18 is below fp64
//     resolution: SURVEY.md §5a)
//   * slacks per advertiser, impressions ascending           R/allocation_mw.cpp:163-171
//   * weights w *= (1+eps)^(s/W) or (1-eps)^(-s/W) as dexp(t * log1p(+-eps)),
//     dexp = round-to-nearest range reduction by ln2 (hi/lo), degree-13 Taylor
//     Horner with fma, ldexp                                 R/allocation_mw.cpp:173-190
//   * averages x_avg = ((t-1)/t) x_avg + (1/t) x             R/instance.cpp:143-152
//
// BINARY mode (R/global_problem.cpp:46-222, 283-292; the mode R/main.cpp:36 runs):
//   * iteration 1: FindMinMaxSlope over regions (impression asc, region asc)
//     with the reference's else-if (a new running maximum is never a minimum
//     candidate), slope_lo = 1/max, slope_hi = 1/min; the interval is
//     [slope_lo, slope_hi] at iteration 1 and [slope_lo*scale, slope_hi/scale]
//     after (slope_lo/hi are never recomputed)      R/global_problem.cpp:116-135, 283-292
//   * one level: d = (upper-lower)/nr, ratio = lower-d, cr_k = (ratio += d);
//     usage_i(r) = sum over regions j (in order) of width_j if u_j >= r;
//     S(r) = sum_blocked(usage) (blocks of 256 impressions, zero padded,
//     halving tree s_l += s_{l+w}, w = 128..1, then sum_fixed of the block
//     sums); delta_k = S(cr_k) - B                       R/global_problem.cpp:137-162
//   * per k: k == 0 and delta < 0 -> lower *= 0.9, next level; k == nr-1 and
//     delta > 0 -> upper /= 0.9, next level; else delta > 0 -> lower = cr_k,
//     delta < 0 -> upper = cr_k and stop the scan, delta == 0 -> allocate at
//     cr_k (all regions u >= cr_k)                        R/global_problem.cpp:66-98
//   * after a level without expansion: stop when upper - lower <
//     max(1e-16, |upper| 2^-42).  The reference's 1e-16 is an x87 long double
//     window of ~925 representable values near 1 (and below fp64 resolution);
//     2^-42 |upper| keeps the same granularity in fp64 (1024..2048 ulp).  A
//     finer fp64 window makes a critical ratio land exactly on a region slope
//     U often (then lower = U and no region is in (lower, upper]: dual 0,
//     which the reference shows only at iteration 1).  At most 2048 levels
//     (the reference recurses without bound when the regions never hold B).
//   * range allocation (lower, upper): regions with u > upper in full
//     (impression asc, region asc), rem = B - sum_blocked(full per
//     impression); then the regions with lower < u <= upper in (impression,
//     region) order: inc = min(rem, width), assigned (beta += inc, j* = j)
//     whatever its sign, rem -= inc, stop when rem == 0   R/global_problem.cpp:180-222
//   * a region assigned with width 0 still sets j* (the reference's make_pair)
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "oracle.h"

namespace {

double sum_fixed(const double* x, int64_t n) {
    double s[64];
    for (int l = 0; l < 64; ++l) {
        double acc = 0.0;
        for (int64_t k = l; k < n; k += 64) acc = acc + x[k];
        s[l] = acc;
    }
    for (int w = 32; w >= 1; w >>= 1)
        for (int l = 0; l < w; ++l) s[l] = s[l] + s[l + w];
    return s[0];
}

double dexp(double x) {
    const double inv_ln2 = 0x1.71547652b82fep+0;
    const double ln2_hi = 0x1.62e42fefa39efp-1;
    const double ln2_lo = 0x1.abc9e3b39803fp-56;
    const double k = std::nearbyint(x * inv_ln2);
    double r = std::fma(-k, ln2_hi, x);
    r = std::fma(-k, ln2_lo, r);
    // 1/j! for j = 13 .. 0
    static const double c[14] = {   // fp64 nearest of 1/13!, 1/12!, ..., 1/1!, 1/0!
        0x1.6124613a86d09p-33, 0x1.1eed8eff8d898p-29, 0x1.ae64567f544e4p-26, 0x1.27e4fb7789f5cp-22,
        0x1.71de3a556c734p-19, 0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-13, 0x1.6c16c16c16c17p-10,
        0x1.1111111111111p-7,  0x1.5555555555555p-5,  0x1.5555555555555p-3, 0x1.0000000000000p-1,
        0x1.0000000000000p+0,  0x1.0000000000000p+0};
    double p = c[0];
    for (int j = 1; j < 14; ++j) p = std::fma(p, r, c[j]);
    return std::ldexp(p, (int)k);
}

// Fixed-order blocked sum of the binary-mode spec: blocks of 256 (zero
// padded), halving tree inside a block, sum_fixed over the block sums.
double sum_blocked(const double* x, int64_t n) {
    const int64_t nb = (n + 255) / 256;
    std::vector<double> bs(nb);
    for (int64_t b = 0; b < nb; ++b) {
        double s[256];
        for (int l = 0; l < 256; ++l) s[l] = (b * 256 + l < n) ? x[b * 256 + l] : 0.0;
        for (int w = 128; w >= 1; w >>= 1)
            for (int l = 0; l < w; ++l) s[l] = s[l] + s[l + w];
        bs[b] = s[0];
    }
    return sum_fixed(bs.data(), nb);
}

constexpr int kMaxLevels = 2048;

struct Pt {
    double p, c;
    int adv;   // -1 for the origin
};

struct Impression {
    int h = 0;                       // hull size (envelope points)
    std::vector<double> u, v, cut;   // h, h, h+1
};

}  // namespace

extern "C" int oracle_mw_run_mode(int A, int I, double sparsity, double scaling, double epsilon,
                                  int T, double tol, int binary, double scale, int intervals,
                                  double* dual, double* infeas, int32_t* infeas_idx, double* wmin,
                                  double* wmax, double* budget_w, double* x_avg_out,
                                  double* weights_out, int64_t* nnz_out, int32_t* levels_out,
                                  double* interval_out) {
    if (binary && (intervals < 1 || intervals > 8 || !(scale > 0.0))) return -2;
    int64_t nnz = 0;
    if (oracle_gen_adalloc(A, I, sparsity, scaling, &nnz, nullptr, nullptr, nullptr, nullptr,
                           nullptr, nullptr) != 0)
        return -1;
    std::vector<int32_t> adv(nnz), imp(nnz), draws(A);
    std::vector<double> bid(nnz), budgets(A);
    double max_bid = 0;
    oracle_gen_adalloc(A, I, sparsity, scaling, &nnz, adv.data(), imp.data(), bid.data(),
                       budgets.data(), draws.data(), &max_bid);
    if (nnz_out) *nnz_out = nnz;
    // impression-major order (impression asc, advertiser asc): position of each bid
    std::vector<int64_t> order(nnz);
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(),
                     [&](int64_t a, int64_t b) { return imp[a] < imp[b]; });
    std::vector<int64_t> iptr(I + 1, 0);
    for (int64_t k = 0; k < nnz; ++k) iptr[imp[k] + 1]++;
    for (int i = 0; i < I; ++i) iptr[i + 1] += iptr[i];
    std::vector<int32_t> i_adv(nnz);
    std::vector<double> i_bid(nnz);
    std::vector<int64_t> pos_of(nnz);   // advertiser-major index -> impression-major index
    for (int64_t q = 0; q < nnz; ++q) {
        i_adv[q] = adv[order[q]];
        i_bid[q] = bid[order[q]];
        pos_of[order[q]] = q;
    }
    // width R/allocation_mw.cpp:154-161 (fp64)
    double width = max_bid * ((double)I * sparsity);
    for (int a = 0; a < A; ++a) width = std::max(width, budgets[a]);
    const double tight_tol = std::max(tol, 1e-12);
    const double lp = std::log1p(epsilon), lm = std::log1p(-epsilon);

    std::vector<double> w(A, 1.0), slack(A, 0.0), avg_slack(A, 0.0);
    std::vector<double> x(nnz, 0.0), xa(nnz, 0.0), wb(A);
    std::vector<Impression> sub(I);
    std::vector<double> dcontrib(I);
    double slope_lo = 0.0, slope_hi = DBL_MAX;   // R/global_problem.cpp:38-39

    for (int t = 1; t <= T; ++t) {
        for (int a = 0; a < A; ++a) wb[a] = w[a] * budgets[a];
        const double B = sum_fixed(wb.data(), A);
        if (budget_w) budget_w[t - 1] = B;
        // ---- subproblems: upper envelope per impression
        for (int i = 0; i < I; ++i) {
            Impression& s = sub[i];
            s.h = 0;
            s.u.clear(); s.v.clear(); s.cut.clear();
            const int64_t b0 = iptr[i], b1 = iptr[i + 1];
            if (b1 == b0) continue;
            std::vector<Pt> P;
            for (int64_t q = b0; q < b1; ++q) P.push_back({i_bid[q], i_bid[q] * w[i_adv[q]], i_adv[q]});
            P.push_back({0.0, 0.0, -1});
            std::sort(P.begin(), P.end(), [](const Pt& a, const Pt& b) {
                if (a.c != b.c) return a.c > b.c;
                if (a.p != b.p) return a.p > b.p;
                return a.adv < b.adv;
            });
            std::vector<Pt> H;
            for (const Pt& q : P) {
                while (H.size() >= 2) {
                    const Pt& O = H[H.size() - 2];
                    const Pt& Aq = H[H.size() - 1];
                    const double d1 = (Aq.c - O.c) * (q.p - O.p);
                    const double d2 = (Aq.p - O.p) * (q.c - O.c);
                    if (d1 - d2 <= 1e-14) H.pop_back(); else break;
                }
                H.push_back(q);
            }
            const int h = (int)H.size();
            s.h = h;
            s.u.push_back(H[h - 2].p / H[h - 2].c);
            s.v.push_back(0.0);
            for (int k = h - 2; k > 0; --k) {
                const double uu = (H[k - 1].p - H[k].p) / (H[k - 1].c - H[k].c);
                s.u.push_back(uu);
                s.v.push_back(H[k - 1].p - H[k - 1].c * uu);
            }
            s.u.push_back(0.0);
            s.v.push_back(H[0].p);
            s.cut.push_back(0.0);
            for (int k = 0; k < h - 1; ++k) {
                if (s.u[k] - s.u[k + 1] > 1e-14)
                    s.cut.push_back((s.v[k + 1] - s.v[k]) / (s.u[k] - s.u[k + 1]));
                else
                    s.cut.push_back(s.cut[k]);
            }
            s.cut.push_back(DBL_MAX);
        }
        std::vector<double> beta(I, 0.0);
        std::vector<int> jstar(I, -1);
        if (binary) {
            // ---- global budget split, binary mode (header)
            const int nr = intervals;
            static const bool trace = std::getenv("ORACLE_MW_TRACE") != nullptr;
            std::vector<double> usage(I);
            auto S = [&](double r, bool strict) {
                for (int i = 0; i < I; ++i) {
                    double acc = 0.0;
                    for (int j = 0; j < sub[i].h - 1; ++j) {
                        const double u = sub[i].u[j];
                        if (strict ? (u > r) : (u >= r)) acc = acc + (sub[i].cut[j + 1] - sub[i].cut[j]);
                    }
                    usage[i] = acc;
                }
                return sum_blocked(usage.data(), I);
            };
            if (t == 1) {
                double maxw = 0.0, minw = DBL_MAX;
                for (int i = 0; i < I; ++i)
                    for (int j = 0; j < sub[i].h - 1; ++j) {
                        const double u = sub[i].u[j];
                        if (u > maxw) maxw = u;
                        else if (u < minw) minw = u;
                    }
                slope_lo = 1.0 / maxw;
                slope_hi = 1.0 / minw;
            }
            double lower = (t == 1) ? slope_lo : slope_lo * scale;
            double upper = (t == 1) ? slope_hi : slope_hi / scale;
            int levels = 0, mode = 0;   // 1 exact (at cr_exact), 2 range (lower, upper)
            double cr_exact = 0.0;
            double cr[8], delta[8];
            for (;;) {
                ++levels;
                const double d = (upper - lower) / (double)nr;
                double r = lower - d;
                for (int k = 0; k < nr; ++k) { r = r + d; cr[k] = r; }
                for (int k = 0; k < nr; ++k) delta[k] = S(cr[k], false) - B;
                if (trace)
                    std::fprintf(stderr, "t=%d level=%d lower=%.17g upper=%.17g d0=%.6g d%d=%.6g\n", t,
                                 levels, lower, upper, delta[0], nr - 1, delta[nr - 1]);
                bool expanded = false;
                for (int k = 0; k < nr; ++k) {
                    if (k == 0 && delta[k] < 0.0) { lower = lower * 0.9; expanded = true; break; }
                    if (k == nr - 1 && delta[k] > 0.0) { upper = upper / 0.9; expanded = true; break; }
                    if (delta[k] > 0.0) lower = cr[k];
                    else if (delta[k] < 0.0) { upper = cr[k]; break; }
                    else { mode = 1; cr_exact = cr[k]; break; }
                }
                if (mode == 1) break;
                if (!expanded && upper - lower < std::max(1e-16, std::fabs(upper) * 0x1p-42)) { mode = 2; break; }
                if (levels >= kMaxLevels) { mode = 2; break; }
            }
            if (levels_out) levels_out[t - 1] = levels;
            if (interval_out) {
                interval_out[2 * (t - 1)] = mode == 1 ? cr_exact : lower;
                interval_out[2 * (t - 1) + 1] = mode == 1 ? cr_exact : upper;
            }
            for (int i = 0; i < I; ++i)
                for (int j = 0; j < sub[i].h - 1; ++j) {
                    const double u = sub[i].u[j];
                    if (mode == 1 ? (u >= cr_exact) : (u > upper)) {
                        beta[i] = beta[i] + (sub[i].cut[j + 1] - sub[i].cut[j]);
                        jstar[i] = j;
                    }
                }
            if (mode == 2) {
                double rem = B - sum_blocked(beta.data(), I);
                bool stop = false;
                for (int i = 0; i < I && !stop; ++i)
                    for (int j = 0; j < sub[i].h - 1; ++j) {
                        const double u = sub[i].u[j];
                        if (u > lower && u <= upper) {
                            const double wd = sub[i].cut[j + 1] - sub[i].cut[j];
                            const double inc = (wd < rem) ? wd : rem;   // std::min(rem, width)
                            beta[i] = beta[i] + inc;
                            jstar[i] = j;
                            rem = rem - inc;
                            if (rem == 0.0) { stop = true; break; }
                        }
                    }
            }
        } else {
        // ---- global budget split, sort mode
        struct Reg { double slope, width; int i, j; };
        std::vector<Reg> regs;
        for (int i = 0; i < I; ++i)
            for (int j = 0; j < sub[i].h - 1; ++j)
                regs.push_back({sub[i].u[j], sub[i].cut[j + 1] - sub[i].cut[j], i, j});
        std::stable_sort(regs.begin(), regs.end(),
                         [](const Reg& a, const Reg& b) { return a.slope > b.slope; });
        const int64_t R = (int64_t)regs.size();
        std::vector<double> pre(R);
        const int64_t C = 256, nch = (R + C - 1) / C;
        std::vector<double> chunk(nch);
        for (int64_t c = 0; c < nch; ++c) {
            double acc = 0.0;
            for (int64_t k = c * C; k < std::min(R, (c + 1) * C); ++k) acc = acc + regs[k].width;
            chunk[c] = acc;
        }
        double off = 0.0;
        for (int64_t c = 0; c < nch; ++c) {
            double acc = off;
            for (int64_t k = c * C; k < std::min(R, (c + 1) * C); ++k) {
                pre[k] = acc;
                acc = acc + regs[k].width;
            }
            off = off + chunk[c];
        }
        for (int64_t k = 0; k < R; ++k) {
            double rem = B - pre[k];
            if (!(rem > 0.0)) rem = 0.0;
            const double inc = std::min(rem, regs[k].width);
            if (inc > 0.0) {
                beta[regs[k].i] = beta[regs[k].i] + inc;
                jstar[regs[k].i] = regs[k].j;
            }
        }
        }
        // ---- primal + dual value
        std::fill(x.begin(), x.end(), 0.0);
        for (int i = 0; i < I; ++i) {
            dcontrib[i] = 0.0;
            if (!(beta[i] > 0.0)) continue;
            const Impression& s = sub[i];
            const double u = s.u[jstar[i]], v = s.v[jstar[i]], bi = beta[i];
            dcontrib[i] = u * bi + v;
            const int64_t b0 = iptr[i], b1 = iptr[i + 1];
            if (u == 0.0) {
                int64_t best = -1;
                double mp = 0.0;
                for (int64_t q = b0; q < b1; ++q)
                    if (mp < i_bid[q]) { mp = i_bid[q]; best = q; }
                if (best >= 0) x[best] = 1.0;
            }
            if (v == 0.0) {
                int64_t best = -1;
                double mr = 0.0;
                for (int64_t q = b0; q < b1; ++q) {
                    const double c = i_bid[q] * w[i_adv[q]];
                    const double r = i_bid[q] / c;
                    if (mr < r) { mr = r; best = q; }
                }
                if (best >= 0) x[best] = bi / (i_bid[best] * w[i_adv[best]]);
            }
            if (u > 0.0 && v > 0.0) {
                int64_t t0 = -1, t1 = -1;
                int nt = 0;
                for (int64_t q = b0; q < b1; ++q) {
                    const double c = i_bid[q] * w[i_adv[q]];
                    double sl = i_bid[q] - (u * c + v);
                    if (sl < 0) sl = -sl;
                    if (sl < tight_tol) {
                        if (nt == 0) t0 = q; else if (nt == 1) t1 = q;
                        ++nt;
                    }
                }
                if (nt == 1) {
                    const double c = i_bid[t0] * w[i_adv[t0]];
                    x[t0] = std::fmin(bi / c, 1.0);
                } else if (nt == 2) {
                    const double c0 = i_bid[t0] * w[i_adv[t0]], c1 = i_bid[t1] * w[i_adv[t1]];
                    const double x1 = (bi - c1) / (c0 - c1);
                    x[t0] = x1;
                    x[t1] = 1.0 - x1;
                }
            }
        }
        dual[t - 1] = sum_fixed(dcontrib.data(), I);
        // ---- averages, slacks, weights
        const double fa = (double)(t - 1) / (double)t, fb = 1.0 / (double)t;
        for (int64_t q = 0; q < nnz; ++q) xa[q] = fa * xa[q] + fb * x[q];
        double worst = 0.0;
        int worst_i = -1;
        double mn = 100000.0, mx = 0.0;   // R/allocation_mw.cpp:254-255
        // slack_a = -B_a + sum over a's bids (impressions ascending) of x * bid
        for (int a = 0; a < A; ++a) slack[a] = -budgets[a];
        for (int64_t k = 0; k < nnz; ++k) slack[adv[k]] = slack[adv[k]] + x[pos_of[k]] * bid[k];
        for (int a = 0; a < A; ++a) {
            avg_slack[a] = fa * avg_slack[a] + fb * slack[a];
            if (avg_slack[a] > 0.0 && avg_slack[a] / budgets[a] > worst) {
                worst = avg_slack[a] / budgets[a];
                worst_i = a;
            }
            const double tt = slack[a] / width;
            w[a] = w[a] * (tt >= 0.0 ? dexp(tt * lp) : dexp(-tt * lm));
            mn = std::min(mn, w[a]);
            mx = std::max(mx, w[a]);
        }
        if (infeas) infeas[t - 1] = worst;
        if (infeas_idx) infeas_idx[t - 1] = worst_i;
        if (wmin) wmin[t - 1] = mn;
        if (wmax) wmax[t - 1] = mx;
    }
    if (x_avg_out) std::memcpy(x_avg_out, xa.data(), sizeof(double) * nnz);
    if (weights_out) std::memcpy(weights_out, w.data(), sizeof(double) * A);
    return 0;
}

extern "C" int oracle_mw_run(int A, int I, double sparsity, double scaling, double epsilon,
                             int T, double tol, double* dual, double* infeas, int32_t* infeas_idx,
                             double* wmin, double* wmax, double* budget_w, double* x_avg_out,
                             double* weights_out, int64_t* nnz_out) {
    return oracle_mw_run_mode(A, I, sparsity, scaling, epsilon, T, tol, 0, 0.0, 0, dual, infeas,
                              infeas_idx, wmin, wmax, budget_w, x_avg_out, weights_out, nnz_out,
                              nullptr, nullptr);
}

extern "C" double oracle_dexp(double x) { return dexp(x); }
extern "C" double oracle_sum_blocked(const double* x, int64_t n) { return sum_blocked(x, n); }
extern "C" double oracle_sum_fixed(const double* x, int64_t n) { return sum_fixed(x, n); }
