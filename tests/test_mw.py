"""f3 — the reference's multiplicative-weights loop (sort mode).

CPU: the fp64 MW spec (oracle/oracle_mw.cpp) tracks the reference's own
long-double run (oracle/_ref/dlp_ref_mw, fixture tests/golden/ref_mw_sort.json):
dual values agree to the reference's printed precision over the first
iterations and within 1e-3 over the whole run (9e-5 at 1000x1000 x 300, 5e-4
at 100x100 x 100), and every dual value bounds the exact OPT from above.
The primal / infeasibility trajectory is not compared: the reference breaks
equal-ratio ties by __gnu_cxx::hash_map iteration order and equal-slope ties by
std::sort internals; the spec fixes both orders.

GPU: the HIP MW path is bit-identical to the fp64 spec, per iteration (dual,
worst infeasibility + advertiser, min / max weight, weighted budget) and in
the final averaged primal and weights."""
import math

import numpy as np
import pytest

import oracle_py as O
from conftest import load_golden

import distributedlpsolver_amd as dlp

REF = load_golden("ref_mw_sort.json")["runs"]
REF_BIN = load_golden("ref_mw_binary.json")["runs"]
OPT = {r["A"]: r["highs_objective"] for r in load_golden("adalloc.json")}


def test_dexp_spec_accuracy():
    xs = np.linspace(-6.0, 6.0, 4001)
    err = max(abs(O.dexp(float(x)) - math.exp(x)) / math.exp(x) for x in xs)
    assert err < 4.5e-16
    assert O.dexp(0.0) == 1.0


def test_sum_fixed_spec():
    O.mw_run(2, 10, 0.5, 0.25, 0.01, 1)   # binds the helpers
    x = np.random.default_rng(0).random(1000)
    s = [0.0] * 64
    for l in range(64):
        acc = 0.0
        for k in range(l, len(x), 64):
            acc = acc + x[k]
        s[l] = acc
    w = 32
    while w >= 1:
        for l in range(w):
            s[l] = s[l] + s[l + w]
        w >>= 1
    assert O.lib().oracle_sum_fixed(x.ctypes.data_as(O._D), len(x)) == s[0]


@pytest.mark.parametrize("key", ["1000x1000", "100x100"])
def test_mw_spec_tracks_reference_dual(key):
    ref = REF[key]
    r = O.mw_run(ref["A"], ref["I"], ref["sparsity"], 0.25, 0.01, ref["iterations"])
    rd = np.array(ref["dual_values"])
    d = r["dual"]
    rel = np.abs(d - rd) / rd
    assert rel[:5].max() < 1e-5                   # the reference prints 6 significant digits
    assert rel.max() < 1e-3                       # tie-order drift (module docstring)
    opt = OPT[ref["A"]]
    assert (d >= opt * (1 - 1e-12)).all()         # MW dual values bound OPT from above
    assert d[-1] > d[0]


@pytest.mark.gpu
@pytest.mark.parametrize("A,I,sp,T", [(2, 10, 0.5, 50), (100, 100, 0.1, 100), (200, 200, 0.1, 60),
                                      (1000, 1000, 0.1, 300)])
def test_mw_gpu_bit_identical_to_spec(A, I, sp, T):
    p = dlp.Problem.adalloc(A, I, 1, sp, 0.25)
    mw = dlp.MW(p)
    log, ms = mw.run(T)
    x, w = mw.solution()
    mw.close()
    r = O.mw_run(A, I, sp, 0.25, 0.01, T)
    np.testing.assert_array_equal(log["dual_value"], r["dual"])
    np.testing.assert_array_equal(log["weighted_budget"], r["budget"])
    np.testing.assert_array_equal(log["max_infeasibility"], r["infeas"])
    np.testing.assert_array_equal(log["infeasible_advertiser"], r["infeas_idx"])
    np.testing.assert_array_equal(log["min_weight"], r["wmin"])
    np.testing.assert_array_equal(log["max_weight"], r["wmax"])
    np.testing.assert_array_equal(w, r["weights"])
    # x: problem variable order (advertiser, impression) vs the oracle's impression-major order
    adv, imp, _ = p.adalloc_bids()
    order = np.lexsort((adv, imp))
    np.testing.assert_array_equal(x[order], r["x_avg"])


@pytest.mark.gpu
def test_mw_gpu_run_in_pieces_equals_one_run():
    p = dlp.Problem.adalloc(100, 100, 1, 0.1, 0.25)
    a = dlp.MW(p)
    la, _ = a.run(40)
    b = dlp.MW(p)
    lb = np.concatenate([b.run(15)[0], b.run(25)[0]])
    assert la.tobytes() == lb.tobytes()
    assert a.solution()[0].tobytes() == b.solution()[0].tobytes()


@pytest.mark.gpu
def test_mw_large_scenario_properties():
    """The reference's commented-out large scenario shape, scaled to a test
    (10k advertisers x 100k impressions x 1e-3): size-independent properties.
    The weighted budget is exactly split (sum of allocations = B when the
    regions suffice), dual values are finite and positive, weights stay
    positive, x >= 0.  (Per-impression sums of x are NOT <= 1: at iteration 1
    all ratios tie and the reference's v == 0 branch gives beta / c to the
    first tied constraint, R/global_problem.cpp:350-365 — reproduced as is.)"""
    A, I = 10000, 100000
    p = dlp.Problem.adalloc(A, I, 1, 1e-3, 0.25)
    mw = dlp.MW(p)
    log, ms = mw.run(20)
    x, w = mw.solution()
    assert np.isfinite(log["dual_value"]).all() and (log["dual_value"] > 0).all()
    assert np.isfinite(x).all() and x.min() >= -1e-6
    assert (w > 0).all() and np.isfinite(w).all()
    # iteration 1: all weights 1 -> B = A * 0.5 * (I // A) * 0.25 exactly, every region has
    # slope 1 and v = 0, so the dual value is the whole budget (the regions hold far more)
    B0 = A * 0.5 * (I // A) * 0.25
    assert log["weighted_budget"][0] == B0
    assert abs(log["dual_value"][0] - B0) <= 1e-9 * B0


# ---------------------------------------------------------------- binary mode
def test_sum_blocked_spec():
    O.mw_run(2, 10, 0.5, 0.25, 0.01, 1)   # binds the helpers
    for n in (0, 1, 255, 256, 257, 1000, 70000):
        x = np.random.default_rng(n).random(n)
        bs = []
        for b in range(0, n, 256):
            s = list(x[b:b + 256]) + [0.0] * (256 - len(x[b:b + 256]))
            w = 128
            while w >= 1:
                for l in range(w):
                    s[l] = s[l] + s[l + w]
                w >>= 1
            bs.append(s[0])
        bs = np.array(bs)
        want = O.lib().oracle_sum_fixed(bs.ctypes.data_as(O._D), len(bs))
        assert O.lib().oracle_sum_blocked(x.ctypes.data_as(O._D), n) == want


def test_mw_scale_is_the_reference_long_double():
    # R/main.cpp:38 in x87 long double, rounded once to fp64
    assert O.mw_scale(0.01) == float(np.longdouble(1) - np.longdouble(0.01) * np.longdouble(0.001))
    assert abs(O.mw_scale(0.01) - (1 - 1e-5)) < 1e-16


@pytest.mark.parametrize("key", ["1000x1000", "100x100"])
def test_mw_binary_spec_tracks_reference(key):
    """Binary (threshold-search) mode, the mode R/main.cpp:36 runs, against the
    reference's own long-double run (tests/golden/ref_mw_binary.json): iteration
    1 prints 0 in both (the search brackets the common slope 1 from above, no
    region lies in (lower, upper]); later duals agree to the printed 6 digits
    over the first iterations and within 1e-3 over the run (tie-order drift, as
    sort mode); the critical intervals agree to the printed digits early on."""
    ref = REF_BIN[key]
    r = O.mw_run(ref["A"], ref["I"], ref["sparsity"], 0.25, 0.01, ref["iterations"], binary=True)
    rd = np.array(ref["dual_values"])
    d = r["dual"]
    assert rd[0] == 0.0 and d[0] == 0.0
    rel = np.abs(d[1:] - rd[1:]) / rd[1:]
    assert rel[:5].max() < 1e-5
    assert rel.max() < 1e-3
    opt = OPT[ref["A"]]
    assert (d[1:] >= opt * (1 - 1e-12)).all()
    cr = np.array(ref["critical_interval"])
    assert np.abs(r["interval"][:10] - cr[:10]).max() <= 1e-5 * np.abs(cr[:10]).max()
    # fp64 stop window: 2^-42 |upper| (or an exact hit)
    lo, up = r["interval"][:, 0], r["interval"][:, 1]
    assert ((up - lo) < np.maximum(1e-16, np.abs(up) * 2.0 ** -42)).all()
    assert (r["levels"] >= 1).all() and (r["levels"] < 2048).all()


def test_mw_binary_intervals_and_scale_are_parameters():
    a = O.mw_run(100, 100, 0.1, 0.25, 0.01, 20, binary=True, intervals=3)
    b = O.mw_run(100, 100, 0.1, 0.25, 0.01, 20, binary=True, intervals=5)
    c = O.mw_run(100, 100, 0.1, 0.25, 0.01, 20, binary=True, scale=1 - 1e-3)
    assert (a["levels"] != b["levels"]).any() and (a["levels"] != c["levels"]).any()
    for r in (a, b, c):   # same optimum bracket within the fp64 window
        assert np.allclose(r["dual"], a["dual"], rtol=1e-9)


def _gpu_vs_spec_binary(A, I, sp, T, **kw):
    p = dlp.Problem.adalloc(A, I, 1, sp, 0.25)
    mw = dlp.MW(p, binary=True, **kw)
    log, ms = mw.run(T)
    x, w = mw.solution()
    mw.close()
    r = O.mw_run(A, I, sp, 0.25, 0.01, T, binary=True, **kw)
    np.testing.assert_array_equal(log["search_levels"], r["levels"])
    np.testing.assert_array_equal(log["dual_value"], r["dual"])
    np.testing.assert_array_equal(log["weighted_budget"], r["budget"])
    np.testing.assert_array_equal(log["max_infeasibility"], r["infeas"])
    np.testing.assert_array_equal(log["infeasible_advertiser"], r["infeas_idx"])
    np.testing.assert_array_equal(log["min_weight"], r["wmin"])
    np.testing.assert_array_equal(log["max_weight"], r["wmax"])
    np.testing.assert_array_equal(w, r["weights"])
    adv, imp, _ = p.adalloc_bids()
    order = np.lexsort((adv, imp))
    np.testing.assert_array_equal(x[order], r["x_avg"])
    return log, ms


@pytest.mark.gpu
@pytest.mark.parametrize("A,I,sp,T", [(2, 10, 0.5, 50), (100, 100, 0.1, 100), (200, 200, 0.1, 60),
                                      (1000, 1000, 0.1, 300)])
def test_mw_gpu_binary_bit_identical_to_spec(A, I, sp, T):
    """One-workgroup search (I <= 16384): bit-identical per iteration, incl. the
    number of search levels."""
    _gpu_vs_spec_binary(A, I, sp, T)


@pytest.mark.gpu
def test_mw_gpu_binary_uncached_and_multi_round_bit_identical_to_spec(monkeypatch):
    """One workgroup, regions read from HBM each level (LDS cache off); and
    1024 < I <= 16384, where each 256-lane group walks several spec blocks."""
    monkeypatch.setenv("DLP_MW_NO_LDS_CACHE", "1")
    _gpu_vs_spec_binary(1000, 1000, 0.1, 20)
    monkeypatch.delenv("DLP_MW_NO_LDS_CACHE")
    _gpu_vs_spec_binary(100, 5000, 0.02, 15)


@pytest.mark.gpu
def test_mw_gpu_binary_multi_launch_bit_identical_to_spec():
    """I > 16384: one launch per search level, last-block reduction + control."""
    _gpu_vs_spec_binary(300, 40000, 0.004, 12)


@pytest.mark.gpu
def test_mw_gpu_binary_parameters():
    _gpu_vs_spec_binary(100, 100, 0.1, 30, intervals=5)
    # one ratio per level never raises `lower` (the reference recurses without
    # bound): every iteration ends at the spec's 2048-level cap
    log, _ = _gpu_vs_spec_binary(100, 100, 0.1, 4, intervals=1, scale=1 - 1e-3)
    assert (log["search_levels"] == 2048).all()


@pytest.mark.gpu
def test_mw_gpu_binary_large_scenario_properties():
    """10k x 100k x 1e-3 in binary mode: iteration 1 is 0 (as the reference),
    later dual values finite and positive, weights positive."""
    p = dlp.Problem.adalloc(10000, 100000, 1, 1e-3, 0.25)
    mw = dlp.MW(p, binary=True)
    log, ms = mw.run(8)
    x, w = mw.solution()
    assert log["dual_value"][0] == 0.0
    assert np.isfinite(log["dual_value"]).all() and (log["dual_value"][1:] > 0).all()
    assert (log["search_levels"] >= 1).all()
    assert np.isfinite(x).all() and (w > 0).all()
