"""CPU, world_size 2-3 over gloo: the product's row-block driver
(distributedlpsolver_amd.rowblock.run_rowblock + dlp_rank_rows) drives
oracle row-slice engines; the multi-rank pivot log must equal the single-rank
log bit for bit (P = 1, 2, 4, 8 logs identical)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_py as O


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, m, n, seed, degenerate, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import distributedlpsolver_amd as dlp
        from distributedlpsolver_amd.rowblock import run_rowblock
        A, b, c = O.gen_dense(m, n, seed, degenerate)
        first, count = dlp.rank_rows(m, rank, world)
        eng = O.OracleEngine(A, b, c, rank, world, first, count)
        status, done = run_rowblock(eng, 100_000)
        log = eng.log()
        q.put((rank, status, done, log.tobytes()))
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,m,n,seed,degenerate", [(2, 40, 60, 1, False), (3, 50, 50, 5, True),
                                                        (2, 64, 64, 5, True), (4, 70, 90, 6, False),
                                                        (4, 48, 64, 7, True)])
def test_rowblock_gloo_matches_single_rank(world, m, n, seed, degenerate):
    A, b, c = O.gen_dense(m, n, seed, degenerate)
    ref = O.solve_dense(A, b, c)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, m, n, seed, degenerate, q))
             for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, status, done, log in out:
        assert status == 0, (rank, status)
        assert done == ref.num_pivots
        got = np.frombuffer(log, O.PIVOT_DTYPE)
        assert got.tobytes() == ref.pivot_log.tobytes()
