#!/usr/bin/env python3
"""f3 measurement: MW iterations/s on the GPU for the reference's scenarios
(R/main.cpp:19-29): default 1000 x 1000 x 0.1 and the (commented-out) large
100000 x 1000000 x 1e-4, in binary (threshold-search) mode, the mode
R/main.cpp:36 runs, and in sort mode.  The reference's own times on one core of
the build container are in BASELINE.md (binary 8.27 s / 300 iterations and
sort 4.91 s at the default; 2.3-2.8 s per iteration relaxation in sort mode at
the large scenario, where its binary mode segfaults).

    python tools/bench_mw.py [--out FILE]
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
ap.add_argument("--large-iterations", type=int, default=30)
ap.add_argument("--only", default=None, help="substring of the case names to run")
a = ap.parse_args()
out = {}
probs = {}
for name, (A, I, sp, T, binary) in {
        "default_1000x1000_binary": (1000, 1000, 0.1, 300, True),
        "default_1000x1000_sort": (1000, 1000, 0.1, 300, False),
        "large_100000x1000000_binary": (100000, 1000000, 1e-4, a.large_iterations, True),
        "large_100000x1000000_sort": (100000, 1000000, 1e-4, a.large_iterations, False)}.items():
    if a.only and a.only not in name:
        continue
    t0 = time.perf_counter()
    if (A, I, sp) not in probs:
        probs.clear()
        probs[(A, I, sp)] = dlp.Problem.adalloc(A, I, 1, sp, 0.25)
    p = probs[(A, I, sp)]
    t1 = time.perf_counter()
    mw = dlp.MW(p, binary=binary)
    t2 = time.perf_counter()
    mw.run(2)                                  # warm-up iterations (not timed)
    t3 = time.perf_counter()
    log, ms = mw.run(T)
    t4 = time.perf_counter()
    rec = dict(A=A, I=I, sparsity=sp, nnz=p.n, iterations=T, host_generate_s=t1 - t0,
               create_s=t2 - t1, device_ms_per_iteration=ms / T,
               wall_ms_per_iteration=1e3 * (t4 - t3) / T, iterations_per_s=T / (t4 - t3),
               mean_search_levels=float(log["search_levels"].mean()),
               final_dual=float(log["dual_value"][-1]),
               final_max_infeasibility=float(log["max_infeasibility"][-1]))
    out[name] = rec
    print(name, json.dumps(rec), flush=True)
    mw.close()
out["reference_cpu_1core"] = {"default_binary_mode_ms_per_iteration": 8270.0 / 300,
                              "default_sort_mode_ms_per_iteration": 4910.0 / 300,
                              "large_sort_mode_relaxation_s_per_iteration": "2.3-2.8",
                              "source": "BASELINE.md / SURVEY.md §6 (build container, 1 core)"}
if a.out:
    json.dump(out, open(a.out, "w"), indent=1)
