"""CPU (gloo, world size 2): bench.py's measurement on N ranks agrees a failure before anyone
moves on.  A rank whose peer-exchange run fails holds its error until every rank has passed the
window's barriers; then all ranks close their sessions and measure again on the reopened (RCCL)
session, or all of them stop.  This is the path a failed xGMI peer run takes in the driver's
scaling bench; here the sessions are stand-ins and the failure is injected."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class ExchangeError(RuntimeError):
    pass


class FakeSession:
    """run() fails once `fail_at` pivots have been asked for on the failing rank."""

    def __init__(self, name, fail_at=None):
        self.name, self.fail_at, self.asked, self.closed, self.resets = name, fail_at, 0, False, 0

    def run(self, pivots):
        self.asked += pivots
        if self.fail_at is not None and self.asked >= self.fail_at:
            raise ExchangeError(f"{self.name}: exchange timeout")
        return 0, pivots

    def reset_timings(self):
        self.resets += 1

    def abort(self):
        self.aborted = True

    def close(self):
        assert getattr(self, "aborted", False), "a failed peer session is aborted and drained before close"
        self.closed = True


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, case, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        warm, timed = 64, 128
        fail_at = {"ok": None, "warm": warm, "timed": warm + timed}[case["fail_in"]]
        first = FakeSession("peer", fail_at if rank == case["fail_rank"] else None)
        opened = []

        def reopen():
            s = FakeSession("rccl", fail_at if case.get("fail_again") and rank == case["fail_rank"] else None)
            opened.append(s)
            return s, "rccl"

        def barrier_sync():
            dist.barrier()

        def any_rank(flag):
            return bench.agree_any(flag, dist, torch, "cpu")

        try:
            sess, st, done, el, why, name = bench.measure_with_fallback(
                first, warm, timed, barrier_sync, any_rank, ExchangeError,
                reopen if case["reopen"] else None)
            q.put((rank, "ok", done, why, name, first.closed, len(opened), sess.resets))
        except SystemExit as e:
            q.put((rank, "exit", str(e), None, None, first.closed, len(opened), 0))
    finally:
        dist.destroy_process_group()


def _run(case, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_no_failure_keeps_the_first_session():
    for rank, kind, done, why, name, closed, nopen, resets in _run(
            {"fail_in": "ok", "fail_rank": -1, "reopen": True}):
        assert kind == "ok" and done == 128 and why is None and name is None
        assert not closed and nopen == 0 and resets == 1


@pytest.mark.parametrize("fail_in", ["warm", "timed"])
def test_one_rank_fails_every_rank_reruns_over_rccl(fail_in):
    """Rank 1 fails (in the warm-up or the timed window); rank 0's run succeeded.  Both ranks
    report the same fallback, close the peer session and time the whole window again."""
    out = _run({"fail_in": fail_in, "fail_rank": 1, "reopen": True})
    for rank, kind, done, why, name, closed, nopen, resets in out:
        assert kind == "ok" and done == 128 and name == "rccl"
        assert why.startswith("peer exchange failed during the run")
        assert ("exchange timeout" in why) == (rank == 1)   # rank 0 only knows another rank failed
        assert closed and nopen == 1 and resets == 1


def test_failure_without_fallback_stops_every_rank():
    out = _run({"fail_in": "timed", "fail_rank": 0, "reopen": False})
    assert [o[1] for o in out] == ["exit", "exit"]
    assert "exchange timeout" in out[0][2] and "another rank" in out[1][2]


def test_fallback_that_fails_again_stops_every_rank():
    out = _run({"fail_in": "warm", "fail_rank": 1, "reopen": True, "fail_again": True})
    assert [o[1] for o in out] == ["exit", "exit"]
    assert all(o[5] and o[6] == 1 for o in out)
