"""General LPs on the GPU: two-phase simplex through
the C ABI against the oracle's restatement (tests/oracle_py.py), bit for bit:
pivot log (Phase I pivots, drive-out pivots, Phase II pivots), x, y, the
objective (NaN when infeasible), the standard-form basis and the Phase I
pivot count.  Multi-rank: P row-block sessions on one GPU exchanged by the
host, and the RCCL exchange path on a 1-rank communicator (the carried
objective row and the forced pivots travel through the same exchange
buffers as ordinary pivots)."""
import numpy as np
import pytest

import oracle_py as O
from conftest import load_golden
from general_lp import INF, fixture_lp, lp_arrays, random_general

import distributedlpsolver_amd as dlp
from distributedlpsolver_amd import _lib as L

pytestmark = pytest.mark.gpu

CASES = load_golden("general.json")


def _same_log(got, ref):
    assert len(got) == len(ref), (len(got), len(ref))
    g, r = np.ascontiguousarray(got), np.ascontiguousarray(ref)
    if g.tobytes() != r.tobytes():
        for k in range(len(r)):
            if g[k].tobytes() != r[k].tobytes():
                raise AssertionError(f"pivot {k}: gpu {g[k]} oracle {r[k]}")


def _check(res, ref, x_too=True):
    assert res.status == ref.status
    _same_log(res.pivot_log, ref.pivot_log)
    assert res.num_pivots == ref.num_pivots
    assert res.phase1_pivots == ref.phase1_pivots
    assert np.float64(res.objective).tobytes() == np.float64(ref.objective).tobytes()
    if x_too:
        assert res.x.tobytes() == ref.x.tobytes()
    assert res.y.tobytes() == ref.y.tobytes()
    assert res.basis.tobytes() == ref.basis.tobytes()


@pytest.mark.parametrize("cs", CASES, ids=[c["name"] for c in CASES])
@pytest.mark.parametrize("pricing", [0, 1])
@pytest.mark.parametrize("defer", [0, 16])  # 0 = auto: eager below 32 MiB
def test_general_fixtures_bit_identical(cs, pricing, defer):
    lp = fixture_lp(cs)
    res = dlp.solve(dlp.Problem.general(*lp_arrays(lp)), pricing=pricing, defer=defer)
    ref = O.solve_general(lp, pricing=pricing)
    _check(res, ref)
    if ref.status == 0 and "highs" in cs and cs["highs"]["status"] == 0:
        h = cs["highs"]["objective"]
        assert abs(res.objective - h) <= 1e-9 * max(1.0, abs(h))


@pytest.mark.parametrize("m,n,seed,sense,frac_eq", [(120, 160, 301, 1, 0.2), (200, 150, 302, -1, 0.3),
                                                    (300, 420, 303, 1, 0.1)])
@pytest.mark.parametrize("defer", [0, 16])  # 0 = auto: eager below 32 MiB
def test_general_random_larger(m, n, seed, sense, frac_eq, defer):
    cs = random_general("r", m, n, seed, sense=sense, c0=0.5, frac_eq=frac_eq)
    lp = fixture_lp(cs)
    res = dlp.solve(dlp.Problem.general(*lp_arrays(lp)), defer=defer)
    ref = O.solve_general(lp, nthreads=8)
    assert ref.status == 0 and ref.phase1_pivots > 0
    _check(res, ref)


@pytest.mark.parametrize("opts", [dict(check_interval=1), dict(check_interval=7, use_graph=0),
                                  dict(check_interval=13, timing=2), dict(update_variant=0),
                                  dict(ld_align=512)])
def test_general_launch_options(opts):
    """The Phase I -> II switch lands anywhere inside a poll window."""
    cs = next(c for c in CASES if c["name"] == "lpgen_2d_20x20_eq")
    lp = fixture_lp(cs)
    res = dlp.solve(dlp.Problem.general(*lp_arrays(lp)), **opts)
    _check(res, O.solve_general(lp))


def test_general_mps_file_solve(tmp_path):
    from general_lp import write_mps
    cs = random_general("r", 40, 50, 305, sense=-1, c0=2.0)
    lp = fixture_lp(cs)
    path = tmp_path / "r.mps"
    want = write_mps(str(path), lp, np.random.default_rng(1))
    res = dlp.solve(dlp.Problem.mps(str(path)))
    ref = O.solve_general(O.GeneralLP(*want))
    _check(res, ref)


def _x_base(lp):
    """x with every standard-form column at 0 (lo, else hi, else 0)."""
    return np.where(np.isfinite(lp.col_lo), lp.col_lo, np.where(np.isfinite(lp.col_hi), lp.col_hi, 0.0))


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("name", ["lpgen_2d_20x20_eq", "random_60x100", "enzo_c_infeasible",
                                  "basic_artificial_vars"])
def test_general_multi_rank_sessions_one_gpu(P, name):
    """P row-block sessions, host exchange: forced drive-out pivots and the
    carried-row switch use the same candidate all-gather / int64 MAX exchange."""
    cs = next(c for c in CASES if c["name"] == name)
    lp = fixture_lp(cs)
    ref = O.solve_general(lp)
    prob = dlp.Problem.general(*lp_arrays(lp))
    sess = [dlp.Session(prob, rank=r, nranks=P) for r in range(P)]
    status = L.RUNNING
    for _ in range(100_000):
        cands = np.concatenate([s.step_candidate() for s in sess])
        sts = {s.status()[0] for s in sess}
        assert len(sts) == 1
        st = sts.pop()
        if st != L.RUNNING:
            status = st
            break
        sends = [s.step_select(cands) for s in sess]
        prow = np.max(np.stack(sends), axis=0)
        for s in sess:
            s.step_update(prow)
    assert status == ref.status
    results = [s.result() for s in sess]
    for r in results:
        _same_log(r.pivot_log, ref.pivot_log)
        assert r.phase1_pivots == ref.phase1_pivots
        assert np.float64(r.objective).tobytes() == np.float64(ref.objective).tobytes()
        assert r.y.tobytes() == ref.y.tobytes()
        assert r.basis.tobytes() == ref.basis.tobytes()
    x = np.sum([r.x for r in results], axis=0) - (P - 1) * _x_base(lp)
    np.testing.assert_allclose(x, ref.x, rtol=0, atol=1e-12 * (1 + np.abs(ref.x).max()))
    # the in-process merge maps every rank's basic rows back to user variables: bit-exact
    merged = dlp.Session.merged_result(sess)
    _check(merged, ref)
    for s in sess:
        s.close()


@pytest.mark.parametrize("name", ["lpgen_2d_20x20_eq", "enzo_c_infeasible", "random_60x100"])
def test_general_solve_n_gpus_in_process(name):
    cs = next(c for c in CASES if c["name"] == name)
    lp = fixture_lp(cs)
    ref = O.solve_general(lp)
    res = dlp.solve(dlp.Problem.general(*lp_arrays(lp)), n_gpus=1, exchange=L.XCHG_RCCL)
    _check(res, ref)


@pytest.mark.parametrize("name", ["lpgen_2d_20x20_eq", "network_flow", "enzo_c_infeasible"])
@pytest.mark.parametrize("defer", [0, 16])  # 0 = auto: eager below 32 MiB
def test_general_rccl_exchange_single_rank(name, defer):
    cs = next(c for c in CASES if c["name"] == name)
    lp = fixture_lp(cs)
    ref = O.solve_general(lp)
    with dlp.Session(dlp.Problem.general(*lp_arrays(lp)), rank=0, nranks=1,
                     rccl_id=dlp.comm_unique_id(), exchange=L.XCHG_RCCL, timing=2, check_interval=5,
                     defer=defer) as s:
        st, _ = s.run(10 ** 6)
        res = s.result()
    assert st == ref.status
    _check(res, ref)


@pytest.mark.parametrize("defer", [0, 8])
def test_general_resume_across_runs(defer):
    """dlp_session_run in small slices (the Phase I end, the drive-out and the
    switch land in different calls) equals one solve."""
    cs = next(c for c in CASES if c["name"] == "random_40x60_max")
    lp = fixture_lp(cs)
    ref = O.solve_general(lp)
    with dlp.Session(dlp.Problem.general(*lp_arrays(lp)), check_interval=3, defer=defer) as s:
        st = L.RUNNING
        while st == L.RUNNING:
            st, _ = s.run(4)
        res = s.result()
    _check(res, ref)


def test_general_infeasible_and_unbounded_status():
    for name, want in (("enzo_c_infeasible", L.INFEASIBLE), ("enzo_c_unbounded", L.UNBOUNDED),
                       ("bounds_equal_but_infeasible", L.INFEASIBLE)):
        cs = next(c for c in CASES if c["name"] == name)
        res = dlp.solve(dlp.Problem.general(*lp_arrays(fixture_lp(cs))))
        assert res.status == want
        if want == L.INFEASIBLE:
            assert np.isnan(res.objective) and not res.y.any()


def test_general_free_rows_and_no_phase1():
    """All-L rows with b >= 0 and x >= 0: no artificials, no carried row, and the
    same pivots as the dense path."""
    A, b, c = O.gen_dense(64, 80, 9)
    dense = dlp.solve(dlp.Problem.dense(A, b, c))
    rl = np.full(65, -INF)
    rh = np.concatenate([b, [INF]])   # plus a free row
    res = dlp.solve(dlp.Problem.general(np.vstack([A, np.ones(80)]), rl, rh, np.zeros(80),
                                        np.full(80, INF), c, 0.0, L.MAXIMIZE))
    assert res.phase1_pivots == 0
    _same_log(res.pivot_log, dense.pivot_log)
    assert res.objective == dense.objective and res.x.tobytes() == dense.x.tobytes()
