"""Failure containment on the RCCL exchange: a rank that fails
ends its peers' waits instead of leaving them blocked behind a collective that
can never complete.  Every case must return the error within a bounded time."""
import os
import threading
import time

import pytest

import oracle_py as O

import distributedlpsolver_amd as dlp
from distributedlpsolver_amd import _lib as L

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("defer", [1, 16])
def test_injected_fault_one_rank_rccl_session(defer):
    A, b, c = O.gen_dense(200, 400, 1)
    with dlp.Session(dlp.Problem.dense(A, b, c), rank=0, nranks=1, rccl_id=dlp.comm_unique_id(), exchange=L.XCHG_RCCL,
                     defer=defer, check_interval=16) as s:
        s.inject_fault(1)   # the second window's wait fails
        t0 = time.time()
        with pytest.raises(L.DLPError) as e:
            s.run(10 ** 6)
        assert e.value.status == L.ERR_RCCL and "injected" in str(e.value)
        assert time.time() - t0 < 30


def test_injected_fault_in_process_n_gpus():
    """dlp_solve(n_gpus = 1): the failing rank's error comes back (the group's
    failure word aborts every communicator of the solve)."""
    A, b, c = O.gen_dense(200, 400, 1)
    os.environ["DLP_TEST_FAIL_RANK"] = "0"
    try:
        t0 = time.time()
        with pytest.raises(L.DLPError) as e:
            dlp.solve(dlp.Problem.dense(A, b, c), n_gpus=1, exchange=L.XCHG_RCCL, check_interval=8, small_lp=-1)
        assert "rank 0" in str(e.value) and "injected" in str(e.value)
        assert time.time() - t0 < 30
    finally:
        del os.environ["DLP_TEST_FAIL_RANK"]
    # the process is healthy afterwards: the same solve succeeds
    res = dlp.solve(dlp.Problem.dense(A, b, c), n_gpus=1, exchange=L.XCHG_RCCL)
    assert res.status == L.OK


def test_abort_from_another_thread():
    """dlp_session_abort while dlp_session_run is waiting on the exchange path."""
    with dlp.Session(dlp.Problem.random(4096, 4096, 2), rank=0, nranks=1, rccl_id=dlp.comm_unique_id(), exchange=L.XCHG_RCCL,
                     check_interval=4096, max_pivots=10 ** 6) as s:
        out = {}

        def run():
            try:
                out["r"] = s.run(10 ** 6)
            except L.DLPError as e:
                out["e"] = e

        th = threading.Thread(target=run)
        t0 = time.time()
        th.start()
        time.sleep(0.5)
        s.abort()
        th.join(timeout=60)
        assert not th.is_alive()
        assert "e" in out and out["e"].status == L.ERR_RCCL and "abort" in str(out["e"])
        assert time.time() - t0 < 60


def test_stall_limit():
    """A window that makes no progress for longer than the exchange timeout is
    aborted (here a 1 ms limit against a 4096-pivot C2 window of ~100 ms)."""
    with dlp.Session(dlp.Problem.random(4096, 4096, 2), rank=0, nranks=1, rccl_id=dlp.comm_unique_id(), exchange=L.XCHG_RCCL,
                     check_interval=4096) as s:
        s.set_exchange_timeout(0.001)
        with pytest.raises(L.DLPError) as e:
            s.run(4096)
        assert e.value.status == L.ERR_RCCL and "exchange timeout" in str(e.value)


@pytest.mark.parametrize("defer", [1, 16])
def test_n_gpus_peer_run_failure_reruns_over_rccl(defer):
    """dlp_solve(n_gpus = 1) with the auto exchange: the peer run fails mid-solve
    (DLP_TEST_FAIL_PEER_RANK injects a failed window wait on the peer exchange only), every
    rank is drained and freed, and the solve is rerun from the start over RCCL.  The result
    is bit-exact and says which exchange produced it and why."""
    A, b, c = O.gen_dense(200, 400, 1)
    ref = O.solve_dense(A, b, c)
    clean = dlp.solve(dlp.Problem.dense(A, b, c), n_gpus=1, defer=defer, check_interval=8, small_lp=-1)
    assert clean.exchange == L.XCHG_PEER and clean.exchange_reason == ""
    os.environ["DLP_TEST_FAIL_PEER_RANK"] = "0"
    try:
        t0 = time.time()
        res = dlp.solve(dlp.Problem.dense(A, b, c), n_gpus=1, defer=defer, check_interval=8, small_lp=-1)
        assert time.time() - t0 < 60
    finally:
        del os.environ["DLP_TEST_FAIL_PEER_RANK"]
    assert res.exchange == L.XCHG_RCCL
    assert "peer exchange failed during the run" in res.exchange_reason and "injected" in res.exchange_reason
    assert res.status == ref.status and res.num_pivots == ref.num_pivots
    assert res.pivot_log.tobytes() == ref.pivot_log.tobytes()
    assert res.x.tobytes() == ref.x.tobytes() and res.y.tobytes() == ref.y.tobytes()
