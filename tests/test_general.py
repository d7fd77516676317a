"""General LPs, CPU side: the oracle's two-phase
restatement against HiGHS fixtures and scipy known answers, the KKT
conditions of its x / y, and the product's host logic (MPS reader, canonical
standard form dimensions, argument validation) through the C ABI without a GPU.

Fixtures: tests/golden/general.json (tests/golden/make_golden.py general):
scipy test_linprog.py KATs restated with citations, the MPS format
description's TESTPROB (tests/golden/testprob.mps) and seeded random general
LPs with every row / column bound type; HiGHS (scipy 1.15.3) objective, x, y.
Tolerances: objective 1e-9 relative (vs HiGHS and vs the scipy known answer),
x 1e-7 where the known answer lists x; y against HiGHS where the duals are
unique (non-degenerate fixtures), else the KKT check below at 1e-7."""
import os

import numpy as np
import pytest

import oracle_py as O
from conftest import GOLDEN, load_golden
from general_lp import INF, fixture_lp, lp_arrays, random_general, write_mps

import distributedlpsolver_amd as dlp
from distributedlpsolver_amd import _lib as L

CASES = load_golden("general.json")
NONUNIQUE_Y = {"network_flow", "network_flow_limited_capacity", "basic_artificial_vars",
               "lpgen_2d_20x20", "lpgen_2d_20x20_eq"}


def close(a, b, rel=1e-9):
    return abs(a - b) <= rel * max(1.0, abs(b))


def kkt_ok(lp, x, y, tol=1e-7):
    """Primal feasibility + sign-correct complementary marginals y (d f / d row bound) and
    reduced costs c - A^T y: proves optimality of x independent of the solver."""
    s = 1.0 if lp.sense == 1 else -1.0
    ax = lp.A @ x
    scale = 1.0 + np.max(np.abs(ax), initial=0.0)
    t = tol * scale
    assert np.all(ax >= lp.row_lo - t) and np.all(ax <= lp.row_hi + t), "row bounds"
    assert np.all(x >= lp.col_lo - t) and np.all(x <= lp.col_hi + t), "column bounds"
    for i in range(lp.m):
        if s * y[i] < -t:
            assert abs(ax[i] - lp.row_hi[i]) <= t, f"row {i}: y < 0 but not at its upper bound"
        if s * y[i] > t:
            assert abs(ax[i] - lp.row_lo[i]) <= t, f"row {i}: y > 0 but not at its lower bound"
    d = lp.c - lp.A.T @ y
    for j in range(lp.n):
        if s * d[j] > t:
            assert abs(x[j] - lp.col_lo[j]) <= t, f"column {j}: d > 0 but not at its lower bound"
        if s * d[j] < -t:
            assert abs(x[j] - lp.col_hi[j]) <= t, f"column {j}: d < 0 but not at its upper bound"
    return True


@pytest.mark.parametrize("cs", CASES, ids=[c["name"] for c in CASES])
@pytest.mark.parametrize("pricing", [0, 1])
def test_oracle_general_vs_highs(cs, pricing):
    lp = fixture_lp(cs)
    s = O.solve_general(lp, pricing=pricing)
    h = cs["highs"]
    assert s.status == h["status"]
    if "expected_status" in cs:
        assert s.status == cs["expected_status"]
    if s.status != 0:
        if s.status == 1:
            assert np.isnan(s.objective)
        return
    assert close(s.objective, h["objective"]), (s.objective, h["objective"])
    if "expected_objective" in cs:
        assert close(s.objective, cs["expected_objective"], 1e-9)
    if "expected_x" in cs:
        np.testing.assert_allclose(s.x, cs["expected_x"], rtol=1e-7, atol=1e-7)
    if cs["name"] not in NONUNIQUE_Y:
        np.testing.assert_allclose(s.x, h["x"], rtol=1e-7, atol=1e-7)
        np.testing.assert_allclose(s.y, h["y"], rtol=1e-7, atol=1e-7)
    assert kkt_ok(lp, s.x, s.y)
    # the objective is the user objective at x
    assert close(s.objective, float(lp.c @ s.x) + lp.c0, 1e-9)


@pytest.mark.parametrize("cs", CASES, ids=[c["name"] for c in CASES])
def test_oracle_general_log_digest(cs):
    """Regression: the oracle's pivot sequence is the committed one."""
    import hashlib
    for pricing in (0, 1):
        s = O.solve_general(fixture_lp(cs), pricing=pricing)
        ref = cs[f"oracle_pricing{pricing}"]
        assert s.num_pivots == ref["pivots"] and s.phase1_pivots == ref["phase1_pivots"]
        assert hashlib.sha256(np.ascontiguousarray(s.pivot_log).tobytes()).hexdigest() == \
            ref["log_sha256"]


@pytest.mark.parametrize("cs", CASES, ids=[c["name"] for c in CASES])
def test_product_standard_form_dims_match_oracle(cs):
    """The product's canonical standard form (host-side, dlp_general.cpp) has the
    dimensions of the oracle's independent restatement."""
    lp = fixture_lp(cs)
    p = dlp.Problem.general(*lp_arrays(lp))
    assert p.std_dims() == O.general_std_dims(lp)
    back = p.to_general()
    for got, want in zip(back[:6], lp_arrays(lp)[:6]):
        assert np.asarray(got).tobytes() == np.asarray(want, dtype=np.float64).tobytes()
    assert back[6] == lp.c0 and back[7] == lp.sense


def test_mps_testprob():
    cs = next(c for c in CASES if c["name"] == "testprob")
    p = dlp.Problem.mps(os.path.join(GOLDEN, "testprob.mps"))
    A, rl, rh, cl, ch, c, c0, sense = p.to_general()
    lp = fixture_lp(cs)
    np.testing.assert_array_equal(A, lp.A)
    np.testing.assert_array_equal(rl, lp.row_lo)
    np.testing.assert_array_equal(rh, lp.row_hi)
    np.testing.assert_array_equal(cl, lp.col_lo)
    np.testing.assert_array_equal(ch, lp.col_hi)
    np.testing.assert_array_equal(c, lp.c)
    assert (c0, sense) == (0.0, L.MINIMIZE)


@pytest.mark.parametrize("seed", [201, 202, 203, 204])
def test_mps_roundtrip_every_section(tmp_path, seed):
    """Random general LPs written as free MPS (OBJSENSE, RANGES on L/G/E rows,
    every bound type, objective constant, free rows) read back exactly."""
    cs = random_general("r", 25, 30, seed, sense=-1 if seed % 2 else 1, c0=1.25 * (seed % 3))
    lp = fixture_lp(cs)
    lp.row_lo[3], lp.row_hi[3] = -INF, INF   # a free row (dropped by the reader)
    lp.col_lo[0], lp.col_hi[0] = 0.0, 1.0    # a BV candidate
    path = tmp_path / "r.mps"
    want = write_mps(str(path), lp, np.random.default_rng(seed))
    got = dlp.Problem.mps(str(path)).to_general()
    for g, w in zip(got[:6], want[:6]):   # values (the generator's -0.0 entries read back as 0.0)
        np.testing.assert_array_equal(g, np.asarray(w, dtype=np.float64))
    assert got[6] == want[6] and got[7] == want[7]


@pytest.mark.parametrize("text,msg", [
    ("NAME X\nROWS\n N OBJ\nCOLUMNS\n    X1 OBJ 1 R9 2\nENDATA\n", "unknown row"),
    ("NAME X\nROWS\n N OBJ\n L R1\nCOLUMNS\n    X1 R1 abc\nENDATA\n", "bad number"),
    ("NAME X\nROWS\n N OBJ\n L R1\nCOLUMNS\n    X1 R1 1\n", "missing ENDATA"),
    ("NAME X\nROWS\n Q R1\nENDATA\n", "bad row type"),
    ("NAME X\nROWS\n N OBJ\n L R1\nCOLUMNS\n    X1 R1 1\nBOUNDS\n SC BND X1 4\nENDATA\n",
     "unsupported bound"),
    ("NAME X\nROWS\n L R1\nCOLUMNS\n    X1 R1 1\nENDATA\n", "no objective"),
])
def test_mps_errors(tmp_path, text, msg):
    path = tmp_path / "bad.mps"
    path.write_text(text)
    with pytest.raises(L.DLPError) as e:
        dlp.Problem.mps(str(path))
    assert e.value.status == L.ERR_ARG and msg in str(e.value)


def test_mps_missing_file():
    with pytest.raises(L.DLPError) as e:
        dlp.Problem.mps("/nonexistent/file.mps")
    assert e.value.status == L.ERR_ARG


def test_mps_markers_repeats_and_objective_constant(tmp_path):
    """Integer MARKER lines are ignored (LP relaxation), repeated entries summed,
    an objective-row RHS v gives c0 = -v, OBJSENSE on the header line."""
    path = tmp_path / "m.mps"
    path.write_text(
        "NAME M\nOBJSENSE MAX\nROWS\n N OBJ\n G R1\nCOLUMNS\n"
        "    MARKER 'MARKER' 'INTORG'\n    X1 OBJ 1 R1 1\n    X1 R1 2\n"
        "    MARKER 'MARKER' 'INTEND'\n    X2 OBJ -1\nRHS\n    RHS OBJ 3.5 R1 2\n"
        "BOUNDS\n UP BND X1 5\n UP X2 -1\nENDATA\n")
    A, rl, rh, cl, ch, c, c0, sense = dlp.Problem.mps(str(path)).to_general()
    np.testing.assert_array_equal(A, [[3.0, 0.0]])
    assert rl[0] == 2.0 and rh[0] == INF
    np.testing.assert_array_equal(cl, [0.0, -INF])   # UP < 0 with lower 0 -> lower -inf
    np.testing.assert_array_equal(ch, [5.0, -1.0])
    np.testing.assert_array_equal(c, [1.0, -1.0])
    assert c0 == -3.5 and sense == L.MAXIMIZE


def test_general_validation():
    A = np.ones((1, 2))
    ok = dict(A=A, row_lo=[-INF], row_hi=[1.0], col_lo=[0, 0], col_hi=[INF, INF], c=[1, 1])
    dlp.Problem.general(**ok)
    for bad in (dict(c=[np.nan, 1]), dict(col_lo=[INF, 0]), dict(row_hi=[np.nan]),
                dict(col_hi=[-INF, INF])):
        with pytest.raises(L.DLPError) as e:
            dlp.Problem.general(**{**ok, **bad})
        assert e.value.status == L.ERR_ARG
    with pytest.raises(L.DLPError) as e:
        dlp.Problem.general(**ok, sense=0)
    assert e.value.status == L.ERR_ARG
    # no constraint rows at all after canonicalisation
    with pytest.raises(L.DLPError) as e:
        dlp.Problem.general(np.zeros((1, 1)), [-INF], [INF], [0.0], [INF], [1.0])
    assert e.value.status == L.ERR_UNSUPPORTED


def test_dense_problem_as_general_has_no_artificials():
    A, b, c = O.gen_dense(20, 30, 1)
    p = dlp.Problem.dense(A, b, c)
    assert p.std_dims() == (20, 50, 50, 0)
    A2, rl, rh, cl, ch, c2, c0, sense = p.to_general()
    q = dlp.Problem.general(A2, rl, rh, cl, ch, c2, c0, sense)
    assert q.std_dims() == (20, 50, 50, 0)   # same canonical tableau as the dense path
    s1 = O.solve_dense(A, b, c)
    s2 = O.solve_general(O.GeneralLP(A2, rl, rh, cl, ch, c2, c0, sense))
    assert s1.pivot_log.tobytes() == s2.pivot_log.tobytes()
    assert s1.objective == s2.objective and s1.x.tobytes() == s2.x.tobytes()
