"""Lookahead: block b+1 is selected on the tableau buffer the
pass of block b reads, replaying block b's sealed steps first, while that pass
writes the other buffer on a second stream.  Every value must stay bit-identical
to the single-buffer deferred path and to the eager path: pivot logs, x, y,
basis and the whole tableau (objective row and padding included), for every
block size, pass form, poll window (windows end inside blocks and drain the
pipeline), termination inside a block (empty blocks copy the tableau), the
RCCL exchange path, and a switch back to the single buffer mid-session."""
import numpy as np
import pytest

import oracle_py as O

import distributedlpsolver_amd as dlp
from distributedlpsolver_amd import _lib as L

pytestmark = pytest.mark.gpu


def _same_log(got, ref):
    assert len(got) == len(ref), (len(got), len(ref))
    g, r = np.ascontiguousarray(got), np.ascontiguousarray(ref)
    if g.tobytes() != r.tobytes():
        for k in range(len(r)):
            if g[k].tobytes() != r[k].tobytes():
                raise AssertionError(f"pivot {k}: gpu {g[k]} oracle {r[k]}")


def _check(res, ref):
    assert res.status == ref.status
    _same_log(res.pivot_log, ref.pivot_log)
    assert np.float64(res.objective).tobytes() == np.float64(ref.objective).tobytes()
    assert res.x.tobytes() == ref.x.tobytes() and res.y.tobytes() == ref.y.tobytes()
    assert res.basis.tobytes() == ref.basis.tobytes()


@pytest.mark.parametrize("K", [2, 5, 8, 16, 32, 64])
@pytest.mark.parametrize("ci", [3, 16, 64, 100])
def test_lookahead_full_solve(K, ci):
    """Full solve (353 pivots) against the oracle; windows of ci pivots, so blocks
    are cut at every offset and the last window runs empty blocks after the optimum."""
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    with dlp.Session(dlp.Problem.dense(A, b, c), defer=K, check_interval=ci, lookahead=1) as s:
        assert s.lookahead()
        st, _ = s.run(10 ** 6)
        res = s.result()
    assert st == L.OK
    _check(res, ref)


@pytest.mark.parametrize("K", [4, 16])
@pytest.mark.parametrize("pricing", [0, 1])
def test_lookahead_degenerate_bland(K, pricing):
    A, b, c = O.gen_dense(128, 128, 3, degenerate=True)
    ref = O.solve_dense(A, b, c, pricing=pricing)
    with dlp.Session(dlp.Problem.dense(A, b, c), defer=K, pricing=pricing, lookahead=1) as s:
        assert s.lookahead()
        s.run(10 ** 6)
        res = s.result()
    _check(res, ref)


@pytest.mark.parametrize("K,rb,nt,form", [(16, 64, 1, 3), (32, 37, 0, 3), (8, 16, 1, 4), (32, 100, 1, 4),
                                          (13, 64, 0, 4), (16, 64, 1, 5), (24, 29, 1, 5),
                                          (32, 256, 1, 20), (16, 64, 0, 20), (5, 7, 1, 3)])
@pytest.mark.parametrize("ci", [45, 13])
def test_lookahead_tableau(K, rb, nt, form, ci):
    """Whole tableau after 45 pivots equals the eager session's, byte for byte."""
    m, n, seed = 300, 520, 5
    prob = dlp.Problem.random(m, n, seed)
    with dlp.Session(prob, defer=1, check_interval=45) as e:
        e.run(45)
        Te = e.tableau()
        le = e.result().pivot_log
    with dlp.Session(prob, defer=K, check_interval=ci, rows_per_block=rb, nontemporal=nt,
                     lookahead=1) as s:
        s.set_defer_tuning(0, form)
        assert s.lookahead()
        s.run(45)
        Td = s.tableau()
        ld = s.result().pivot_log
    _same_log(ld, le)
    assert Td.tobytes() == Te.tobytes()


@pytest.mark.parametrize("form,rb,nt,ci", [(21, 256, 1, 64), (21, 37, 0, 100), (3, 64, 1, 64), (21, 1000, 1, 30),
                                            (22, 256, 1, 64), (22, 37, 0, 100), (23, 256, 1, 64), (23, 37, 0, 100),
                                            (23, 1000, 1, 30), (23, 768, 1, 64)])
def test_lookahead_k64_tableau(form, rb, nt, ci):
    """K = 64 under lookahead: selections replay up to 127 steps (the sealed block in
    flight + their own), the 128-step ratio kernel; two full blocks and a partial one,
    windows ending inside blocks; whole tableau byte-equal to the eager session's."""
    m, n, seed = 700, 1337, 7
    k = 2 * 64 + 17
    prob = dlp.Problem.random(m, n, seed)
    with dlp.Session(prob, defer=1, check_interval=k) as e:
        e.run(k)
        Te = e.tableau()
        le = e.result().pivot_log
    with dlp.Session(prob, defer=64, check_interval=ci, rows_per_block=rb, nontemporal=nt,
                     lookahead=1) as s:
        s.set_defer_tuning(0, form)
        assert s.lookahead()
        done = 0
        while done < k:
            done += s.run(min(ci, k - done))[1]
        Td = s.tableau()
        ld = s.result().pivot_log
    _same_log(ld, le)
    assert Td.tobytes() == Te.tobytes()


def test_lookahead_medium_tableau_and_auto_policy():
    """2049 x 4097 doubles (75 MB, K = 16): auto leaves lookahead off (K = 64 streaming only); forced
    on, the same pivots and tableau rows as off.  (Auto-on at full size: test_gpu_large's
    C3 tests.)"""
    prob = dlp.Problem.random(2048, 2048, 2)
    with dlp.Session(prob, check_interval=100) as c:
        assert not c.lookahead()
    with dlp.Session(prob, check_interval=100, lookahead=1) as a, dlp.Session(
            prob, check_interval=100, lookahead=0) as b:
        assert a.lookahead() and not b.lookahead()
        assert a.update_stats()[2] == 16 and b.update_stats()[2] == 16
        a.run(300)
        b.run(300)
        _same_log(a.result().pivot_log, b.result().pivot_log)
        rows = [0, 1, 777, 2047, 2048]
        assert a.read_rows(0, 2049)[rows].tobytes() == b.read_rows(0, 2049)[rows].tobytes()


def test_lookahead_unbounded():
    A = np.array([[1.0, -1.0], [-1.0, 0.0]])
    b = np.array([1.0, 0.0])
    c = np.array([1.0, 1.0])
    with dlp.Session(dlp.Problem.dense(A, b, c), defer=8, lookahead=1) as s:
        st, _ = s.run(100)
        assert st == L.UNBOUNDED


def test_lookahead_then_step_api():
    """The step API turns lookahead off (drain, single buffer) and continues the solve."""
    m, n, seed = 150, 170, 4
    A, b, c = O.gen_dense(m, n, seed)
    ref = O.solve_dense(A, b, c)
    prob = dlp.Problem.random(m, n, seed)
    with dlp.Session(prob, defer=8, check_interval=11, lookahead=1) as s:
        assert s.lookahead()
        s.run(37)
        for _ in range(10_000):
            cands = s.step_candidate()
            st, _ = s.status()
            if st != L.RUNNING:
                break
            s.step_update(s.step_select(cands))
        assert not s.lookahead()
        res = s.result()
    _same_log(res.pivot_log, ref.pivot_log)
    assert np.float64(res.objective).tobytes() == np.float64(ref.objective).tobytes()


def test_lookahead_off_for_streamed_form():
    """Retuning to a pass form without an out-of-place instance ends lookahead; the
    solve carries on bit-identically."""
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    with dlp.Session(dlp.Problem.dense(A, b, c), defer=16, check_interval=20, lookahead=1) as s:
        s.run(50)
        assert s.lookahead()
        s.set_defer_tuning(0, 6)
        assert not s.lookahead()
        s.run(10 ** 6)
        res = s.result()
    _check(res, ref)


@pytest.mark.parametrize("defer,form", [(8, -1), (32, -1), (64, 21), (64, 3), (64, 22), (64, 23)])
def test_lookahead_rccl_exchange_single_rank(defer, form):
    """The RCCL path (candidate all-gather, select, MAX all-reduce, commit) with the
    pass on the second stream, as bench.py --gpus N runs it (K = 64: the LEAN
    selection kernels of the multi-GPU C3 geometry, 128-step replays)."""
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    with dlp.Session(dlp.Problem.dense(A, b, c), rank=0, nranks=1, rccl_id=dlp.comm_unique_id(), exchange=L.XCHG_RCCL,
                     defer=defer, check_interval=40, lookahead=1) as s:
        if form >= 0:
            s.set_defer_tuning(0, form)
        assert s.lookahead()
        st, _ = s.run(10 ** 6)
        res = s.result()
    assert st == L.OK
    _check(res, ref)


def test_lookahead_pass_timing():
    """timing = 1: the pass events sit on the pass stream; one pass per block."""
    prob = dlp.Problem.random(300, 520, 5)
    with dlp.Session(prob, defer=16, check_interval=64, timing=1, lookahead=1) as s:
        s.run(64)
        launches, ms, K = s.update_stats()
        assert K == 16 and launches == 4 and ms > 0
