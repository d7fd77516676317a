"""CPU: pin the oracle (tests/oracle_py.py -> oracle/liboracle.so) before it
is trusted as the parity checker: known-answer LPs, HiGHS fixtures, the
generator spec, and the reference's own generated instance."""
import hashlib

import numpy as np
import pytest

import oracle_py as O
from conftest import load_golden


def _log_rows(log):
    return [[int(e["q"]), int(e["p"]), int(e["leaving"]), float(e["ratio"]), float(e["objective"])]
            for e in log]


@pytest.mark.parametrize("kat", load_golden("kat.json"), ids=lambda k: k["name"])
@pytest.mark.parametrize("pricing", [0, 1])
def test_kat(kat, pricing):
    s = O.solve_dense(np.array(kat["A"]), np.array(kat["b"]), np.array(kat["c"]), pricing=pricing)
    exp_status = kat.get("expected_status", 0)
    assert s.status == exp_status
    if exp_status == 0:
        np.testing.assert_allclose(s.objective, kat.get("expected_objective",
                                                        kat.get("highs", {}).get("objective")),
                                   rtol=1e-12)
        if "expected_x" in kat:
            np.testing.assert_allclose(s.x, kat["expected_x"], atol=1e-12)
    if "expected_pivots" in kat:
        assert s.num_pivots == kat["expected_pivots"]
    # regression golden of the oracle's own pivot sequence
    assert s.num_pivots == kat[f"oracle_pivots_pricing{pricing}"]
    assert _log_rows(s.pivot_log) == kat[f"oracle_log_pricing{pricing}"]


def test_beale_cycles_without_bland():
    """Pure Dantzig with lowest-index ties cycles on Beale's LP;
    the hybrid rule switches to Bland after a degenerate pivot and terminates."""
    kat = [k for k in load_golden("kat.json") if k["name"] == "beale_cycling"][0]
    A, b, c = np.array(kat["A"]), np.array(kat["b"]), np.array(kat["c"])
    hybrid = O.solve_dense(A, b, c, pricing=0)
    assert hybrid.status == 0 and hybrid.num_pivots <= 10
    degenerate = (hybrid.pivot_log["ratio"] == 0).sum()
    assert degenerate >= 4


@pytest.mark.parametrize("case", [c for c in load_golden("generated.json")
                                  if c["m"] * c["n"] <= 128 * 128 or c["name"].startswith("c1")],
                         ids=lambda c: c["name"])
def test_generated_vs_highs(case):
    A, b, c = O.gen_dense(case["m"], case["n"], case["seed"], case["degenerate"])
    head = case["gen_head"]
    assert [float(v) for v in A[0, :8]] == head["A00_07"]
    assert [float(v) for v in b[:4]] == head["b0_3"]
    assert [float(v) for v in c[:4]] == head["c0_3"]
    assert float(np.sum(b)) == head["b_sum"]
    s = O.solve_dense(A, b, c)
    assert s.status == 0
    hi = case["highs"]
    assert abs(s.objective - hi["objective"]) <= 1e-9 * abs(hi["objective"])
    if not case["degenerate"]:
        np.testing.assert_allclose(s.x, hi["x"], rtol=1e-9, atol=1e-9)
        np.testing.assert_allclose(s.y, hi["y"], rtol=1e-9, atol=1e-9)
    assert s.num_pivots == case["oracle"]["pivots"]
    assert hashlib.sha256(np.ascontiguousarray(s.pivot_log).tobytes()).hexdigest() == \
        case["oracle"]["log_sha256"]


def test_generated_degenerate_256x512():
    case = [c for c in load_golden("generated.json") if c["name"] == "c4_degen_256x512_s4"][0]
    A, b, c = O.gen_dense(case["m"], case["n"], case["seed"], True)
    s = O.solve_dense(A, b, c, nthreads=8)
    assert s.status == 0
    assert abs(s.objective - case["highs"]["objective"]) <= 1e-9 * case["highs"]["objective"]
    assert s.num_pivots == case["oracle"]["pivots"]
    assert (s.pivot_log["ratio"] == 0).sum() == case["oracle"]["degenerate_pivots"]


def test_tableau_generator_matches_dense_generator():
    m, n, seed = 37, 53, 11
    for degen in (False, True):
        A, b, c = O.gen_dense(m, n, seed, degen)
        T = O.gen_tableau(m, n, seed, degen)
        N = n + m
        assert T.shape == (m + 1, O.ld(m, n))
        np.testing.assert_array_equal(T[:m, :n], A)
        np.testing.assert_array_equal(T[:m, N], b)
        np.testing.assert_array_equal(T[:m, n:N], np.eye(m))
        np.testing.assert_array_equal(T[m, :n], -c)
        assert not T[:, N + 1:].any() and not T[m, n:].any()
        # row slices are slices
        Ts = O.gen_tableau(m, n, seed, degen, row_first=10, row_count=7)
        np.testing.assert_array_equal(Ts[:7], T[10:17])
        np.testing.assert_array_equal(Ts[7], T[m])


def test_degenerate_family_shape():
    A, b, c = O.gen_dense(400, 50, 9, degenerate=True)
    cone = b == 0
    assert 0.4 < cone.mean() < 0.6
    assert (A[cone] < 0).any() and (A[~cone] >= 0).all()


@pytest.mark.parametrize("rec", load_golden("adalloc.json"), ids=lambda r: f"{r['A']}x{r['I']}")
def test_adalloc_generator(rec):
    g = O.gen_adalloc(rec["A"], rec["I"], rec["sparsity"], rec["scaling"])
    assert len(g["bid"]) == rec["nnz"]
    assert sorted(set(int(d) for d in g["draws"])) == rec["draws_per_advertiser"]
    assert float(g["budgets"][0]) == rec["budget"]
    assert hashlib.sha256(g["bid"].tobytes()).hexdigest() == rec["bids_sha256"]


def test_adalloc_generator_matches_reference_binary_output():
    """Degrees printed by the reference itself (oracle/_ref/dlp_ref, built from
    its own sources, R/instance.cpp:178-185) equal the restated generator's."""
    ref = load_golden("ref_adalloc_1000.json")
    g = O.gen_adalloc(1000, 1000, 0.1, 0.25)
    adv_deg = np.bincount(g["adv"], minlength=1000)
    imp_deg = np.bincount(g["imp"], minlength=1000)
    assert adv_deg.tolist() == ref["advertiser_degrees"]
    assert imp_deg.tolist() == ref["impression_degrees"]


@pytest.mark.parametrize("A,I", [(2, 10), (100, 100), (200, 200)])
def test_adalloc_lp_oracle_vs_highs(A, I):
    rec = [r for r in load_golden("adalloc.json") if (r["A"], r["I"]) == (A, I)][0]
    M, b, c = O.adalloc_lp(A, I, rec["sparsity"], rec["scaling"])
    s = O.solve_dense(M, b, c)
    assert s.status == 0
    assert abs(s.objective - rec["highs_objective"]) <= 1e-9 * rec["highs_objective"]


def test_mw_dual_values_bound_opt():
    """The reference's MW "Dual Value" is an upper bound on OPT (SURVEY.md §0
    decision 3): iterations 2..300 of its binary-mode run are >= OPT (125.0);
    iteration 1 prints 0 (its threshold allocation fails), a known exception."""
    ref = load_golden("ref_adalloc_1000.json")
    opt = [r for r in load_golden("adalloc.json") if r["A"] == 1000][0]["highs_objective"]
    dual = ref["dual_values"]
    assert len(dual) == 300
    assert all(d >= opt * (1 - 1e-6) for d in dual[1:])


def test_slices_equal_single_rank():
    """Row-block protocol inside the oracle: P simulated ranks, manual
    all-gather / max all-reduce, same pivot log as P = 1."""
    A, b, c = O.gen_dense(60, 80, 3)
    ref = O.solve_dense(A, b, c)
    for P in (2, 3, 5):
        m = 60
        bounds = [(m * r) // P for r in range(P + 1)]
        eng = [O.OracleEngine(A, b, c, r, P, bounds[r], bounds[r + 1] - bounds[r])
               for r in range(P)]
        for _ in range(10_000):
            cands = np.concatenate([e.step_candidate() for e in eng])
            if eng[0].status()[0] != 4:
                break
            sends = [e.step_select(cands) for e in eng]
            prow = np.max(np.stack(sends), axis=0)
            for e in eng:
                e.step_update(prow)
        logs = [e.log() for e in eng]
        for lg in logs:
            assert lg.tobytes() == ref.pivot_log.tobytes()
        for e in eng:
            e.close()


def test_c5_batch_digests_reproduce():
    """tests/golden/digests.json c5 (the GPU test compares all 4,096 LPs against it): the
    64 x 64 batch re-solved here by the oracle gives the committed per-field digests."""
    import hashlib
    import numpy as np
    g = load_golden("digests.json")["c5"]["64x64"]
    st, npiv, obj, basis, h = [], [], [], [], hashlib.sha256()
    for k in range(g["nlp"]):
        A, b, c = O.gen_dense(64, 64, g["seed"] + k)
        r = O.solve_dense(A, b, c, nthreads=1)
        st.append(r.status)
        npiv.append(r.num_pivots)
        obj.append(r.objective)
        basis.append(r.basis)
        h.update(np.ascontiguousarray(r.pivot_log[:64]).tobytes())
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert sha(np.asarray(st, np.int32)) == g["status_sha256"]
    assert sha(np.asarray(npiv, np.int64)) == g["num_pivots_sha256"]
    assert sha(np.asarray(obj, np.float64)) == g["objective_sha256"]
    assert sha(np.asarray(basis, np.int32)) == g["basis_sha256"]
    assert h.hexdigest() == g["log64_sha256"]


def test_c4_degen_digest_reproduces():
    """tests/golden/digests.json c4_degen_2048x4096 (the GPU test checks the whole tableau against
    it): the oracle re-run here to the first stop gives the committed digests."""
    import hashlib
    g = load_golden("digests.json")["c4_degen_2048x4096"]
    first = min(int(k) for k in g["stops"])
    want = g["stops"][str(first)]
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    got = {}

    def at(k, T, log, basis):
        h = hashlib.sha256()
        for r in range(0, T.shape[0], 512):
            h.update(np.ascontiguousarray(T[r:r + 512, :g["width"]]).tobytes())
        got.update(log=sha(log), basis=sha(basis), tableau=h.hexdigest(), obj=float(log[-1]["objective"]).hex(),
                   degen=int((log["ratio"] == 0.0).sum()))

    O.run_generated_stops(g["m"], g["n"], g["seed"], [first], at, degenerate=True, nthreads=8)
    assert got == {"log": want["log_sha256"], "basis": want["basis_sha256"], "tableau": want["tableau_sha256"],
                   "obj": want["objective_hex"], "degen": want["degenerate_pivots"]}


@pytest.mark.parametrize("m,n,seed,K,k,degen", [(150, 170, 4, 16, 10 ** 6, False), (150, 170, 4, 64, 10 ** 6, False),
                                                (96, 128, 6, 7, 10 ** 6, True), (300, 420, 11, 64, 200, False),
                                                (300, 420, 11, 1, 77, False)])
def test_deferred_oracle_equals_eager(m, n, seed, K, k, degen):
    """oracle/oracle_defer.inc (the GPU's deferred rank-K algorithm on the CPU, bench.py's
    like-for-like CPU baseline) against the eager oracle: pivot log, basis and the whole
    tableau byte for byte, for full solves (optimal inside a block) and windows that end
    inside a block (the last partial block's pass applied)."""
    lg_d, T_d, b_d = O.run_generated_defer(m, n, seed, K, k, degenerate=degen, nthreads=4)
    rows = np.arange(m + 1, dtype=np.int64)
    lg_e, T_e, b_e = O.run_generated(m, n, seed, k, rows, degenerate=degen, nthreads=4)
    assert len(lg_d) == len(lg_e) > 0
    assert np.ascontiguousarray(lg_d).tobytes() == np.ascontiguousarray(lg_e).tobytes()
    assert b_d.tobytes() == b_e.tobytes()
    assert T_d.tobytes() == T_e.tobytes()


def test_deferred_oracle_bench_windows():
    """The like-for-like CPU baseline's windows: whole blocks, every one applied."""
    runs, gen = O.bench_windows_defer(400, 600, 11, 16, [(2, 64, 30.0), (1, 32, 30.0)], gen_threads=2)
    assert runs[0][1] == 64 and runs[1][1] == 32 and all(s > 0 for s, _ in runs) and gen > 0
