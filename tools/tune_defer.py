#!/usr/bin/env python3
"""Interleaved A/B of deferred rank-k configurations on an HBM-resident tableau.

    python tools/tune_defer.py [--workload c3|c2] [--ks 8,16,32] [--rbs 32,64,128]
        [--occs 0,2,4] [--nts 1] [--blocks 4] [--rounds 3] [--out file.json]

One session per block size K (the same LP each), every config (K, rows per
band, workgroups/CU cap, nt) runs `blocks` x K real pivots per round, configs
shuffled per round, all in one process on one device.  Reports per-pivot wall
time (host clock around dlp_session_run, synchronised), pivots/s, and the
tableau pass's per-launch time and GB/s of algorithmic bytes 16 m_local (N+1)."""
import argparse
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributedlpsolver_amd as dlp  # noqa: E402

W = {"c3": (32768, 32768, 3), "c2": (4096, 4096, 2)}
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c3", choices=sorted(W))
ap.add_argument("--ks", default="8,16,32")
ap.add_argument("--rbs", default="32,64,128")
ap.add_argument("--occs", default="0,2,4")
ap.add_argument("--nts", default="1")
ap.add_argument("--forms", default="2")
ap.add_argument("--fused", default="1", help="fused single-rank pivot launch: 0, 1 or 0,1")
ap.add_argument("--blocks", type=int, default=4)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--timing", type=int, default=2)
ap.add_argument("--window", type=int, default=0,
                help="pivots per timed window (0 = blocks x K); < K times one partial-block pass")
ap.add_argument("--out", default=None)
a = ap.parse_args()
m, n, seed = W[a.workload]
sess = {}
for K in map(int, a.ks.split(",")):
    s = dlp.Session(dlp.Problem.random(m, n, seed), timing=a.timing, defer=K,
                    check_interval=K * a.blocks, max_pivots=10 ** 7, log_pivots=0)
    s.run(K)
    sess[K] = s
    print(f"session K={K} ready", flush=True)
any_s = next(iter(sess.values()))
bytes_pass = 16.0 * any_s.rows * (any_s.ncols + 1)
cfgs = [(K, rb, occ, nt, fm, fu) for K in sess for rb in map(int, a.rbs.split(","))
        for occ in map(int, a.occs.split(",")) for nt in map(int, a.nts.split(","))
        for fm in map(int, a.forms.split(",")) for fu in map(int, a.fused.split(","))
        if not (fm in (0, 4, 6, 7, 10, 11, 14, 15, 16, 17) and K > 32)]
res = {c: {"wall": [], "pass": []} for c in cfgs}
rng = random.Random(0)
for r in range(a.rounds):
    order = cfgs[:]
    rng.shuffle(order)
    for c in order:
        K, rb, occ, nt, fm, fu = c
        s = sess[K]
        s.set_tuning(22, rb, nt)
        s.set_defer_tuning(occ, fm)
        s.set_fused_pivot(bool(fu))
        s.run(K)   # first window after a retune (graph rebuild) is not timed
        s.reset_timings()
        s.status()
        win = a.window or K * a.blocks
        t0 = time.perf_counter()
        s.run(win)
        s.status()
        dt = time.perf_counter() - t0
        nl, ms, _ = s.update_stats()
        res[c]["wall"].append(dt * 1e3 / win)
        if nl:
            res[c]["pass"].append(ms / nl)
    print(f"round {r} done", flush=True)
rows = []
for c, v in res.items():
    w = statistics.median(v["wall"])
    p = statistics.median(v["pass"]) if v["pass"] else float("nan")
    rows.append(dict(K=c[0], rows_per_block=c[1], occupancy=c[2], nontemporal=c[3], form=c[4], fused=c[5],
                     ms_per_pivot=w, pivots_per_s=1e3 / w, pass_ms=p,
                     pass_gbs=bytes_pass / p / 1e6 if p == p else None))
rows.sort(key=lambda d: d["ms_per_pivot"])
for d in rows:
    print(f"K={d['K']:2d} rb={d['rows_per_block']:4d} occ={d['occupancy']} nt={d['nontemporal']} "
          f"form={d['form']} fused={d['fused']}  "
          f"{d['ms_per_pivot']:.4f} ms/pivot  {d['pivots_per_s']:.0f} pivots/s  "
          f"pass {d['pass_ms']:.3f} ms  {d['pass_gbs'] or 0:.0f} GB/s")
if a.out:
    json.dump(dict(workload=a.workload, m=m, n=n, bytes_per_pass=bytes_pass, rounds=a.rounds,
                   blocks=a.blocks, timing=a.timing, results=rows), open(a.out, "w"), indent=1)
