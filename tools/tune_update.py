#!/usr/bin/env python3
"""Interleaved A/B of rank-1 update configurations on HBM-resident tableaus.

    python tools/tune_update.py [--workload c3|c2] [--rounds 3] [--pivots 10]
        [--variants 0,7,12] [--rbs 8,16] [--nts 1] [--ld-aligns 16,512]

A config is (row alignment, variant, rows_per_block, nontemporal).  One session
per row alignment (the same LP each), every config runs `pivots` real pivots per
round, configs shuffled per round, all in ONE process on ONE device
(cdna_hip_programming.md §5.4 rule 24).  Reports median/min update-kernel ms
(HIP events) and GB/s of algorithmic bytes 16 (m_local+1)(N+1)."""
import argparse
import json
import os
import random
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributedlpsolver_amd as dlp  # noqa: E402

W = {"c3": (32768, 32768, 3), "c2": (4096, 4096, 2)}
ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c3", choices=sorted(W))
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--pivots", type=int, default=10)
ap.add_argument("--variants", default="0,7,12")
ap.add_argument("--rbs", default="0,8,16")
ap.add_argument("--nts", default="1")
ap.add_argument("--ld-aligns", default="16")
ap.add_argument("--out", default=None)
a = ap.parse_args()
m, n, seed = W[a.workload]
sessions = {}
for al in map(int, a.ld_aligns.split(",")):
    s = dlp.Session(dlp.Problem.random(m, n, seed), timing=1, check_interval=max(a.pivots, 1),
                    max_pivots=10 ** 7, log_pivots=0, ld_align=al, defer=1)
    s.run(3)
    sessions[al] = s
cfgs = [(al, v, rb, nt) for al in sessions for v in map(int, a.variants.split(","))
        for rb in map(int, a.rbs.split(",")) for nt in map(int, a.nts.split(","))]
res = {c: [] for c in cfgs}
any_s = next(iter(sessions.values()))
bytes_launch = 16.0 * (any_s.rows + 1) * (any_s.ncols + 1)
rng = random.Random(0)
for r in range(a.rounds):
    order = cfgs[:]
    rng.shuffle(order)
    for c in order:
        s = sessions[c[0]]
        s.set_tuning(c[1], c[2], c[3])
        s.run(1)            # first launch after a retune is not timed
        s.reset_timings()
        s.run(a.pivots)
        tm, ns = s.timings()
        res[c].append(tm[3] / max(ns, 1))
    print(f"round {r} done", flush=True)
rows = []
for c, v in res.items():
    med, mn = statistics.median(v), min(v)
    rows.append(dict(ld_align=c[0], variant=c[1], rows_per_block=c[2], nontemporal=c[3],
                     median_ms=med, min_ms=mn, median_gbs=bytes_launch / med / 1e6,
                     best_gbs=bytes_launch / mn / 1e6))
rows.sort(key=lambda d: d["median_ms"])
for d in rows:
    print(f"al={d['ld_align']:4d} v{d['variant']:<2d} rb={d['rows_per_block']:4d} nt={d['nontemporal']}  "
          f"median {d['median_ms']:.4f} ms  {d['median_gbs']:.0f} GB/s  (best {d['best_gbs']:.0f})")
if a.out:
    json.dump(dict(workload=a.workload, m=m, n=n, bytes_per_launch=bytes_launch, rounds=a.rounds,
                   pivots=a.pivots, results=rows), open(a.out, "w"), indent=1)
