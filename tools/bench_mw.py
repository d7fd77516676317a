#!/usr/bin/env python3
"""f3 measurement: MW iterations/s on the GPU for the reference's scenarios
(R/main.cpp:19-29): default 1000 x 1000 x 0.1 and the (commented-out) large
100000 x 1000000 x 1e-4.  The reference's own sort-mode times on one core of
the build container are in BASELINE.md (4.91 s / 300 iterations at the default;
2.3-2.8 s per iteration relaxation at the large scenario).

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
a = ap.parse_args()
out = {}
for name, (A, I, sp, T) in {"default_1000x1000": (1000, 1000, 0.1, 300),
                            "large_100000x1000000": (100000, 1000000, 1e-4, a.large_iterations)}.items():
    t0 = time.perf_counter()
    p = dlp.Problem.adalloc(A, I, 1, sp, 0.25)
    t1 = time.perf_counter()
    mw = dlp.MW(p)
    t2 = time.perf_counter()
    mw.run(2)                                  # warm-up iterations (not timed)
    t3 = time.perf_counter()
    log, ms = mw.run(T)
    t4 = time.perf_counter()
    rec = dict(A=A, I=I, sparsity=sp, nnz=p.n, iterations=T, host_generate_s=t1 - t0,
               create_s=t2 - t1, device_ms_per_iteration=ms / T,
               wall_ms_per_iteration=1e3 * (t4 - t3) / T, iterations_per_s=T / (t4 - t3),
               final_dual=float(log["dual_value"][-1]),
               final_max_infeasibility=float(log["max_infeasibility"][-1]))
    out[name] = rec
    print(name, json.dumps(rec), flush=True)
    mw.close()
out["reference_cpu_1core"] = {"default_sort_mode_ms_per_iteration": 4910.0 / 300,
                              "large_sort_mode_relaxation_s_per_iteration": "2.3-2.8",
                              "source": "BASELINE.md / SURVEY.md §6 (build container, 1 core)"}
if a.out:
    json.dump(out, open(a.out, "w"), indent=1)
