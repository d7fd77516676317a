#!/usr/bin/env python3
"""Full solves of small / degenerate LPs at several deferred block sizes K
(1 = eager rank-1), interleaved, to set the auto K for cache-resident tableaus.

    python tools/tune_small_defer.py [--ks 1,4,8,16] [--rounds 3]

Every K gives the same pivot sequence (bit-identical by construction); only
wall time differs.  Prints microseconds per pivot per (LP, K)."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributedlpsolver_amd as dlp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ks", default="1,4,8,16")
ap.add_argument("--rounds", type=int, default=3)
a = ap.parse_args()
lps = {"C4 degenerate 256x512": dlp.Problem.random(256, 512, 4, degenerate=True),
       "C4 degenerate 1024x2048": dlp.Problem.random(1024, 2048, 4, degenerate=True),
       "C1 dense 200x400": dlp.Problem.random(200, 400, 1),
       "dense 1024x1024": dlp.Problem.random(1024, 1024, 7)}
ks = [int(k) for k in a.ks.split(",")]
best = {}
for r in range(a.rounds):
    for name, prob in lps.items():
        for K in ks:
            t0 = time.perf_counter()
            res = dlp.solve(prob, defer=K)
            dt = time.perf_counter() - t0
            key = (name, K)
            us = 1e6 * dt / max(res.num_pivots, 1)
            best[key] = min(best.get(key, 1e30), us)
            if r == 0 and K == ks[0]:
                print(f"{name}: {res.num_pivots} pivots, status {res.status}", flush=True)
for name in lps:
    print(name, "  ".join(f"K={K}: {best[(name, K)]:.1f} us/pivot" for K in ks), flush=True)
