"""Row-block multi-rank pivot driver over a host-side communicator.

The production multi-GPU path runs the whole pivot loop natively with RCCL
(``Session(..., rccl_id=...)`` -> ``dlp_session_run``).  This module drives the
SAME per-rank steps through ``torch.distributed`` instead (gloo on the host, or
any backend that takes CPU tensors), one exchange per pivot:

    candidate  = engine.step_candidate()            local pricing + ratio test
    gathered   = all_gather(candidate)               P x 32 B
    prow_send  = engine.step_select(gathered)        same winner on every rank;
                                                     owner: pivot-row fp64 bits,
                                                     others: INT64_MIN
    prow       = all_reduce(prow_send, MAX)          exact owner bits everywhere
    engine.step_update(prow)                         local rank-1 elimination

It replaces the reference's "distribution layer" (independent per-impression
subproblems coordinated by a scalar budget split, R/global_problem.cpp:270-274,
R/allocation_mw.cpp:271-326) with a row partition of one tableau
(SURVEY.md §8e).  Rows of rank r: ``rank_rows(m, r, P)``.

Engines: ``SessionEngine`` (libdlp on a GPU) here; tests add a CPU checker
engine with the same three methods to check the protocol without a GPU.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import _lib as L
from .solver import CAND_DTYPE, Problem, Session


class SessionEngine:
    """One rank of a libdlp row-block session driven by a host communicator."""

    def __init__(self, problem: Problem, rank: int, nranks: int, **opts):
        self.session = Session(problem, rank=rank, nranks=nranks, rccl_id=None, **opts)

    def step_candidate(self) -> np.ndarray:
        return self.session.step_candidate()

    def step_select(self, gathered: np.ndarray) -> np.ndarray:
        return self.session.step_select(gathered)

    def step_update(self, prow_bits: np.ndarray) -> None:
        self.session.step_update(prow_bits)

    def status(self) -> tuple[int, int]:
        return self.session.status()


def _all_gather_cands(cand: np.ndarray, group=None) -> np.ndarray:
    world = dist.get_world_size(group)
    send = torch.from_numpy(np.frombuffer(cand.tobytes(), dtype=np.uint8).copy())
    recv = [torch.empty(32, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(recv, send, group=group)
    raw = b"".join(t.numpy().tobytes() for t in recv)
    return np.frombuffer(raw, dtype=CAND_DTYPE).copy()


def _all_reduce_max(bits: np.ndarray, group=None) -> np.ndarray:
    t = torch.from_numpy(np.ascontiguousarray(bits, dtype=np.int64).copy())
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return t.numpy()


def run_rowblock(engine, max_pivots: int, group=None) -> tuple[int, int]:
    """Drive ``max_pivots`` pivots; returns (status, pivots done).

    Every rank reaches every decision from identical replicated data (objective
    row, basis, gathered candidates), so all ranks leave the loop together.
    """
    status = L.RUNNING
    for _ in range(max_pivots):
        cand = engine.step_candidate()
        st, _ = engine.status()
        if st != L.RUNNING:
            status = st
            break
        gathered = _all_gather_cands(cand, group)
        prow_send = engine.step_select(gathered)
        st, _ = engine.status()
        if st != L.RUNNING:
            status = st
            break
        engine.step_update(_all_reduce_max(prow_send, group))
    else:
        status = L.PIVOT_LIMIT
    _, done = engine.status()
    return status, done
