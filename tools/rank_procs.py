#!/usr/bin/env python3
"""Diagnostics: P rank sessions of one generated LP as P processes on this GPU (IPC peer exchange over
gloo-gathered handles, as tests/test_gpu_ranks.py), W pivots, each rank's status / pivots / seconds.

    python tools/rank_procs.py M N SEED P PIVOTS [KEY=VALUE env ...]"""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, world, port, m, n, seed, pivots, env, q):
    import torch.distributed as dist
    os.environ.update(env)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import distributedlpsolver_amd as dlp
    out = {"rank": rank}
    s = None
    try:
        la = int(env.get("LOOKAHEAD", "-1"))
        s = dlp.Session(dlp.Problem.random(m, n, seed), rank=rank, nranks=world, defer=0, lookahead=la,
                        check_interval=pivots, max_pivots=pivots + 2)
        hs = [None] * world
        dist.all_gather_object(hs, s.exchange_handle())
        s.connect_ipc(hs)
        s.set_exchange_timeout(float(env.get("XTIMEOUT", "30")))
        out["config"] = {"lookahead": s.lookahead(), "chain_cus": s.chain_cus(),
                         "defer_tuning": s.get_defer_tuning(), "rows": s.rows}
        dist.barrier()
        t0 = time.time()
        try:
            out["run"] = s.run(pivots)
        except Exception as e:  # noqa: BLE001
            out["run_error"] = str(e)
        out["seconds"] = time.time() - t0
        s.abort()
        import torch
        torch.cuda.synchronize()
        dist.barrier()
        s.close()
        s = None
    except Exception as e:  # noqa: BLE001
        out["error"] = repr(e)
    finally:
        q.put(out)
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    m, n, seed, world, pivots = (int(a) for a in sys.argv[1:6])
    env = dict(a.split("=", 1) for a in sys.argv[6:])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = [ctx.Process(target=worker, args=(r, world, port, m, n, seed, pivots, env, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = sorted((q.get(timeout=300) for _ in procs), key=lambda o: o["rank"])
    for p in procs:
        p.join(timeout=60)
        if p.exitcode is None:
            p.kill()
    print(json.dumps({"m": m, "n": n, "P": world, "pivots": pivots, "env": env, "ranks": outs}), flush=True)


if __name__ == "__main__":
    main()
