#!/usr/bin/env python3
"""Per-phase pivot timing (HIP events, timing=2) and wall-clock pivots/s with
hipGraph windows (timing=0) for a few sizes.

    python tools/phase_timing.py [--out FILE]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributedlpsolver_amd as dlp  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--out", default=None)
a = ap.parse_args()
cases = [("c1_200x400", 200, 400, 1, False, 300), ("c4_2048x4096_degen", 2048, 4096, 4, True, 1000),
         ("c2_4096x4096", 4096, 4096, 2, False, 500), ("m1024_n1024", 1024, 1024, 7, False, 1000)]
out = {}
for name, m, n, seed, degen, k in cases:
    rec = {}
    with dlp.Session(dlp.Problem.random(m, n, seed, degen), timing=2, check_interval=k) as s:
        s.run(5)
        s.reset_timings()
        s.run(k)
        tm, ns = s.timings()
        rec["phase_us"] = {p: 1e3 * tm[i] / max(ns, 1) for i, p in
                           enumerate(["ratio", "exchange", "prow", "update"])}
        rec["pivots_timed"] = ns
    for graph in (1, 0):
        with dlp.Session(dlp.Problem.random(m, n, seed, degen), timing=0, check_interval=k,
                         use_graph=graph) as s:
            s.run(k)            # first window captures / warms
            t0 = time.perf_counter()
            st, done = s.run(k)
            dt = time.perf_counter() - t0
        rec[f"wall_us_per_pivot_graph{graph}"] = 1e6 * dt / max(done, 1)
        rec[f"pivots_graph{graph}"] = done
    out[name] = rec
    print(name, json.dumps(rec), flush=True)
if a.out:
    json.dump(out, open(a.out, "w"), indent=1)
