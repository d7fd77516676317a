"""GPU: the owner-rooted peer exchange (include/dlp.h "peer exchange", DESIGN.md §5;
VERDICT r02 #4).  Instead of an RCCL all-gather of the 32-B candidates and an
int64 MAX all-reduce of the 528 KB pivot row, every rank stores its candidate into
every rank's exchange block and the pivot-row owner stores its row into every
rank's block, each message followed by a flag the select / commit kernels wait
for (bounded).  This replaces the reference's distribution layer
(R/global_problem.cpp:270-274) on the row-block partition of SURVEY.md §8(e).

On one GPU the ranks are sessions of one process on the same device (same-device
pointers, dlp_sessions_connect + dlp_sessions_run) or two processes on the same
device (IPC handles of the exchange blocks, dlp_session_connect_ipc).  Every case
is compared with the oracle bit for bit (pivot log, objective, x, y) — the
exchange moves bits and never changes a decision."""
import os
import socket
import time

import numpy as np
import pytest

import oracle_py as O
from conftest import load_golden, tableau_sha256
from general_lp import fixture_lp, lp_arrays

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
    assert res.x.tobytes() == ref.x.tobytes()
    assert res.y.tobytes() == ref.y.tobytes()
    np.testing.assert_array_equal(res.basis, ref.basis)


def _peer_ranks(prob, P, **opts):
    sess = [dlp.Session(prob, rank=r, nranks=P, **opts) for r in range(P)]
    dlp.Session.connect_peers(sess)
    assert all(s.get_exchange() == L.XCHG_PEER for s in sess)
    return sess


@pytest.mark.parametrize("P,K,form", [(2, 1, -1), (3, 1, -1), (8, 1, -1), (2, 16, -1), (3, 32, -1),
                                      (4, 16, -1), (8, 16, -1), (2, 64, 21), (4, 64, 21), (8, 64, 21),
                                      (4, 64, 23), (8, 64, -1)])
def test_peer_exchange_dense(P, K, form):
    m, n, seed = 150, 170, 4
    A, b, c = O.gen_dense(m, n, seed)
    ref = O.solve_dense(A, b, c)
    sess = _peer_ranks(dlp.Problem.random(m, n, seed), P, defer=K, check_interval=37)
    try:
        if form >= 0:
            for s in sess:
                s.set_defer_tuning(0, form)
        st, done = dlp.Session.run_ranks(sess, 10 ** 6)
        assert st == L.OK and done == ref.num_pivots
        _check(dlp.Session.merged_result(sess), ref)
        for s in sess:   # every rank's replicated log and objective row
            r = s.result()
            _same_log(r.pivot_log, ref.pivot_log)
            assert r.y.tobytes() == ref.y.tobytes()
    finally:
        for s in sess:
            s.close()


@pytest.mark.parametrize("P,K", [(3, 1), (2, 16)])
def test_peer_exchange_degenerate_bland(P, K):
    """Degenerate LP (Bland after degenerate pivots, exact ties on the ratio)."""
    A, b, c = O.gen_dense(96, 128, 6, True)
    ref = O.solve_dense(A, b, c)
    sess = _peer_ranks(dlp.Problem.random(96, 128, 6, True), P, defer=K)
    try:
        st, _ = dlp.Session.run_ranks(sess, 10 ** 6)
        assert st == ref.status
        _check(dlp.Session.merged_result(sess), ref)
    finally:
        for s in sess:
            s.close()


@pytest.mark.parametrize("P,K", [(2, 1), (3, 16), (4, 16), (2, 64)])
def test_peer_exchange_unbounded(P, K):
    """An unbounded LP through the peer exchange: column 5 of A small and non-positive with
    c_5 = 0.5, so x_5 enters after 96 pivots, no row bounds it, and every rank's selection ends
    the solve DLP_UNBOUNDED at the same pivot as the oracle (every rank's candidates empty).
    K = 64: with lookahead forced on, the end comes in the second block's selection while the
    first block's pass runs."""
    A, b, c = O.gen_dense(60, 80, 9)
    A[:, 5] = -np.abs(A[:, 5]) * 0.01
    c[5] = 0.5
    ref = O.solve_dense(A, b, c)
    assert ref.status == L.UNBOUNDED and ref.num_pivots == 96
    sess = _peer_ranks(dlp.Problem.dense(A, b, c), P, defer=K, check_interval=29,
                       lookahead=1 if K == 64 else -1)
    try:
        assert all(s.lookahead() for s in sess) == (K == 64)
        st, done = dlp.Session.run_ranks(sess, 10 ** 6)
        assert st == L.UNBOUNDED and done == ref.num_pivots
        for s in sess:
            r = s.result()
            assert r.status == L.UNBOUNDED
            _same_log(r.pivot_log, ref.pivot_log)
    finally:
        for s in sess:
            s.close()


def test_peer_exchange_lookahead_and_windows():
    """Lookahead forced on (selection of block b+1 beside pass b) and windows that end
    inside blocks, resumed: the peer sequence numbers continue across runs."""
    A, b, c = O.gen_dense(150, 170, 4)
    ref = O.solve_dense(A, b, c)
    sess = _peer_ranks(dlp.Problem.random(150, 170, 4), 2, defer=16, lookahead=1, check_interval=7)
    try:
        assert all(s.lookahead() for s in sess)
        total = 0
        while True:
            st, done = dlp.Session.run_ranks(sess, 23)
            total += done
            if st != L.PIVOT_LIMIT and st != L.RUNNING:
                break
        assert st == L.OK and total == ref.num_pivots
        _check(dlp.Session.merged_result(sess), ref)
    finally:
        for s in sess:
            s.close()


@pytest.mark.parametrize("P,form", [(2, 21), (4, 21), (3, 23)])
def test_peer_exchange_lookahead_k64(P, form):
    """Lookahead forced on at K = 64 with the peer exchange: the LEAN selection kernels
    (LDS-DMA rings) push candidates and pivot rows to the peers while the pass of the
    sealed block runs, and read rows of finished bands from the pass's output (band
    publication, form 21; form 23 replays every row).  Windows end inside blocks."""
    m, n, seed = 400, 600, 11
    A, b, c = O.gen_dense(m, n, seed)
    ref = O.solve_dense(A, b, c)
    assert ref.num_pivots > 3 * 64
    sess = _peer_ranks(dlp.Problem.random(m, n, seed), P, defer=64, lookahead=1, check_interval=64)
    try:
        for s in sess:
            s.set_defer_tuning(0, form)
        assert all(s.lookahead() for s in sess)
        total = 0
        while True:
            st, done = dlp.Session.run_ranks(sess, 101)
            total += done
            if st != L.PIVOT_LIMIT and st != L.RUNNING:
                break
        assert st == L.OK and total == ref.num_pivots
        _check(dlp.Session.merged_result(sess), ref)
    finally:
        for s in sess:
            s.close()


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("name", ["lpgen_2d_20x20_eq", "enzo_c_infeasible", "basic_artificial_vars"])
def test_peer_exchange_general(P, name):
    """General LPs: forced drive-out pivots and the carried Phase II objective row
    travel through the same exchange blocks."""
    cs = next(c for c in load_golden("general.json") if c["name"] == name)
    lp = fixture_lp(cs)
    ref = O.solve_general(lp)
    sess = _peer_ranks(dlp.Problem.general(*lp_arrays(lp)), P)
    try:
        st, _ = dlp.Session.run_ranks(sess, 10 ** 6)
        assert st == ref.status
        res = dlp.Session.merged_result(sess)
        _same_log(res.pivot_log, ref.pivot_log)
        assert res.phase1_pivots == ref.phase1_pivots
        assert np.float64(res.objective).tobytes() == np.float64(ref.objective).tobytes()
        assert res.x.tobytes() == ref.x.tobytes() and res.y.tobytes() == ref.y.tobytes()
    finally:
        for s in sess:
            s.close()


@pytest.mark.parametrize("defer", [1, 16])
def test_solve_n_gpus_peer_exchange(defer):
    """dlp_solve(n_gpus = 1, exchange = PEER): the in-process multi-device path
    with the peer exchange instead of the RCCL collectives."""
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    res = dlp.solve(dlp.Problem.dense(A, b, c), n_gpus=1, defer=defer, exchange=L.XCHG_PEER, small_lp=-1)
    _check(res, ref)


@pytest.mark.parametrize("defer", [1, 16])
def test_rccl_session_switches_exchange(defer):
    """A 1-rank RCCL session: set_exchange(PEER) all-gathers the IPC handles over its
    communicator; switching back and forth between windows keeps the result exact."""
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    with dlp.Session(dlp.Problem.dense(A, b, c), rank=0, nranks=1, rccl_id=dlp.comm_unique_id(),
                     defer=defer, check_interval=16, exchange=L.XCHG_PEER) as s:
        assert s.get_exchange() == L.XCHG_PEER
        s.run(50)
        s.set_exchange(L.XCHG_RCCL)
        s.run(50)
        s.set_exchange(L.XCHG_PEER)
        st, _ = s.run(10 ** 6)
        assert st == L.OK
        _check(s.result(), ref)


@pytest.mark.parametrize("inject", [False, True])
@pytest.mark.parametrize("defer", [1, 16])
def test_auto_exchange_rank_session(inject, defer):
    """exchange = DLP_XCHG_DEFAULT (auto) on a 1-rank RCCL session: the ranks agree on the
    peer exchange when every one can make and open the blocks; a rank that cannot
    (DLP_TEST_PEER_FAIL injects it) makes every rank fall back to RCCL, with the reason
    reported.  Bit-exact either way."""
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    if inject:
        os.environ["DLP_TEST_PEER_FAIL"] = "0"
    try:
        s = dlp.Session(dlp.Problem.dense(A, b, c), rank=0, nranks=1, rccl_id=dlp.comm_unique_id(),
                        defer=defer, check_interval=16, small_lp=-1)
    finally:
        os.environ.pop("DLP_TEST_PEER_FAIL", None)
    with s:
        if inject:
            assert s.get_exchange() == L.XCHG_RCCL
            assert "injected" in s.exchange_reason() and "rank 0" in s.exchange_reason()
        else:
            assert s.get_exchange() == L.XCHG_PEER and s.exchange_reason() == ""
        st, _ = s.run(10 ** 6)
        assert st == L.OK
        _check(s.result(), ref)


@pytest.mark.parametrize("lookahead", [0, 1])
def test_peer_one_launch_pivot(lookahead):
    """DLP_PEER_ONELAUNCH=1: the peer pivot as ONE launch (the ratio workgroups publish the
    selection record to the pivot-row workgroups of the same launch); bit-exact on a 1-rank
    exchange session, with K = 64 blocks through lookahead (the LEAN instance) and without."""
    m, n, seed = 400, 600, 11
    A, b, c = O.gen_dense(m, n, seed)
    ref = O.solve_dense(A, b, c)
    os.environ["DLP_PEER_ONELAUNCH"] = "1"
    try:
        with dlp.Session(dlp.Problem.random(m, n, seed), rank=0, nranks=1, rccl_id=dlp.comm_unique_id(),
                         defer=64, lookahead=lookahead, check_interval=50) as s:
            assert s.get_exchange() == L.XCHG_PEER and s.lookahead() == bool(lookahead)
            st, _ = s.run(10 ** 6)
            assert st == L.OK
            _check(s.result(), ref)
    finally:
        os.environ.pop("DLP_PEER_ONELAUNCH", None)


def test_strict_peer_exchange_fails_when_a_rank_cannot():
    """exchange = DLP_XCHG_PEER is not downgraded: the session creation fails."""
    A, b, c = O.gen_dense(64, 64, 3)
    os.environ["DLP_TEST_PEER_FAIL"] = "0"
    try:
        with pytest.raises(L.DLPError) as e:
            dlp.Session(dlp.Problem.dense(A, b, c), rank=0, nranks=1, rccl_id=dlp.comm_unique_id(),
                        exchange=L.XCHG_PEER)
        assert e.value.status == L.ERR_UNSUPPORTED and "injected" in str(e.value)
    finally:
        os.environ.pop("DLP_TEST_PEER_FAIL", None)


@pytest.mark.parametrize("inject", [False, True])
def test_solve_n_gpus_auto_exchange(inject):
    """dlp_solve(n_gpus = 1) with the default exchange: peer, or RCCL after a failed
    connect (injected); bit-exact either way."""
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    if inject:
        os.environ["DLP_TEST_PEER_FAIL"] = "0"
    try:
        res = dlp.solve(dlp.Problem.dense(A, b, c), n_gpus=1, defer=16, small_lp=-1)
    finally:
        os.environ.pop("DLP_TEST_PEER_FAIL", None)
    _check(res, ref)


def test_peer_wait_is_bounded():
    """A rank that never runs: the other rank's select kernel waits for its
    candidate; the host stall limit raises the abort word, the device wait ends and
    the run returns an error instead of hanging."""
    prob = dlp.Problem.random(120, 150, 4)
    sess = _peer_ranks(prob, 2, defer=1)
    try:
        sess[0].set_exchange_timeout(2.0)
        t0 = time.time()
        with pytest.raises(L.DLPError) as e:
            sess[0].run(100)   # rank 1 never enqueues anything
        assert e.value.status == L.ERR_RCCL
        assert time.time() - t0 < 30
    finally:
        for s in sess:
            s.close()


@pytest.mark.parametrize("lookahead", [-1, 0])
def test_c3_row_partition_peer_exchange_one_gpu(lookahead):
    """BASELINE.json C3 (32768 x 32768) as the 8-GPU split runs it, on ONE MI355X:
    8 rank sessions (4,096 local rows each; K = 64, 256-row bands), the exchange through
    the peer blocks, 160 pivots (two full blocks + a 32-pivot tail), against the
    oracle's committed digests: pivot log, basis, objective and the whole tableau.
    lookahead -1 (auto): once connected by the peer exchange every rank selects block b+1
    beside the form-21 pass of block b (band publication on); 0: no
    lookahead, the form-23 pass."""
    g = load_golden("digests.json")
    tab = g["c3_tableau"]
    k, P = 160, 8
    want = tab["stops"][str(k)]
    prob = dlp.Problem.random(tab["m"], tab["n"], tab["seed"])
    sess = [dlp.Session(prob, rank=r, nranks=P, defer=64, check_interval=64, lookahead=lookahead)
            for r in range(P)]
    try:
        on = lookahead != 0
        for s in sess:
            assert s.get_defer_tuning()[1:] == (23, 64) and s.get_tuning()[1] == 256
            assert not s.lookahead()   # a host-driven rank until connected
        dlp.Session.connect_peers(sess)
        for s in sess:
            assert s.lookahead() == on and s.get_defer_tuning()[1] == (21 if on else 23)
        st, done = dlp.Session.run_ranks(sess, k)
        assert done == k
        for s in sess:
            lg = s.result().pivot_log
            assert len(lg) == k
            import hashlib
            assert hashlib.sha256(np.ascontiguousarray(lg).tobytes()).hexdigest() == want["log_sha256"]
        merged = dlp.Session.merged_result(sess)
        import hashlib
        assert hashlib.sha256(np.ascontiguousarray(merged.basis).tobytes()).hexdigest() == want["basis_sha256"]
        assert float(merged.objective).hex() == want["objective_hex"]
        assert tableau_sha256(sess, tab["width"]) == want["tableau_sha256"]
    finally:
        for s in sess:
            s.close()


# ---- two processes on one GPU: IPC handles of the exchange blocks ---------------------

def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ipc_worker(rank, world, port, m, n, seed, defer, q, late=0.0):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s = dlp.Session(dlp.Problem.random(m, n, seed), rank=rank, nranks=world, defer=defer,
                        check_interval=29)
        hs = [None] * world
        dist.all_gather_object(hs, s.exchange_handle())
        s.connect_ipc(hs)
        s.set_exchange_timeout(60.0)
        if rank == world - 1 and late > 0:
            time.sleep(late)   # a rank whose run starts late: its peers' device waits hold
        st, done = s.run(10 ** 6)
        res = s.result()
        q.put((rank, st, done, np.ascontiguousarray(res.pivot_log).tobytes(), res.objective,
               res.x.tobytes(), res.y.tobytes()))
        dist.barrier()   # no rank frees its block while a peer may still read it
        s.close()
    except Exception as e:   # reported to the parent, which fails the test
        q.put((rank, "error", repr(e), None, None, None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("defer,late", [(1, 0.0), (16, 0.0), (16, 32.0)])
def test_peer_exchange_two_processes_ipc(defer, late):
    """late = 32 s: the last rank starts its run 32 s after the first; the first rank's
    device waits are bounded by its exchange timeout (60 s + 5 s), not by a fixed limit of
    their own (round 3 had 30 s), so the solve completes."""
    import torch.multiprocessing as mp
    m, n, seed, world = 120, 150, 4, 2
    A, b, c = O.gen_dense(m, n, seed)
    ref = O.solve_dense(A, b, c)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ipc_worker, args=(r, world, port, m, n, seed, defer, q, late))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=110) for _ in procs]
    for p in procs:
        p.join(timeout=30)
    for rank, st, done, log, obj, x, y in out:
        assert st != "error", done
        assert st == L.OK and done == ref.num_pivots
        assert log == np.ascontiguousarray(ref.pivot_log).tobytes()
        assert obj == ref.objective and y == ref.y.tobytes()
    xs = np.sum([np.frombuffer(o[5]) for o in out], axis=0)
    assert xs.tobytes() == ref.x.tobytes()
    assert all(p.exitcode == 0 for p in procs)
