#!/usr/bin/env python3
"""Secondary measurements (not the bench.py headline): full solves of the
small / degenerate configs, the C5 batch, and the reference's own generated
instance, each next to the CPU oracle (same pivot rule) on this host.

    python tools/bench_extra.py [--out FILE] [--threads 16]

Rows (BASELINE.json configs):
  C1   200 x 400 dense, seed 1, solved to optimality
  C4   degenerate 256 x 512 (seed 4), 2048 x 4096 pivot window
  C5   4096 independent 64 x 64 LPs, one LDS-resident workgroup each
  f1   the reference's default scenario (R/main.cpp:19-38): 1000 advertisers x
       1000 impressions x sparsity 0.1 -> LP 2000 x 96068, solved exactly
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import distributedlpsolver_amd as dlp  # noqa: E402
import oracle_py as O  # noqa: E402  (CPU comparator only)

ap = argparse.ArgumentParser()
ap.add_argument("--out", default=None)
ap.add_argument("--threads", type=int, default=16)
a = ap.parse_args()
out = {}


def timed(fn):
    t0 = time.perf_counter()
    r = fn()
    return r, time.perf_counter() - t0


# warm the device / library
dlp.solve(dlp.Problem.random(16, 16, 1))

# C1: full solve (host-supplied data), GPU vs oracle
A, b, c = O.gen_dense(200, 400, 1)
p = dlp.Problem.dense(A, b, c)
res, t_gpu = timed(lambda: dlp.solve(p))
ref, t_cpu = timed(lambda: O.solve_dense(A, b, c, nthreads=1))
assert np.ascontiguousarray(res.pivot_log).tobytes() == np.ascontiguousarray(ref.pivot_log).tobytes()
out["c1_full_solve"] = dict(pivots=res.num_pivots, gpu_s=t_gpu, gpu_us_per_pivot=1e6 * t_gpu / res.num_pivots,
                            cpu_oracle_s_1thread=t_cpu, objective=res.objective)

# C4 degenerate 256 x 512 full solve
A, b, c = O.gen_dense(256, 512, 4, degenerate=True)
p = dlp.Problem.dense(A, b, c)
res, t_gpu = timed(lambda: dlp.solve(p))
ref, t_cpu = timed(lambda: O.solve_dense(A, b, c, nthreads=1))
assert np.ascontiguousarray(res.pivot_log).tobytes() == np.ascontiguousarray(ref.pivot_log).tobytes()
out["c4_degenerate_256x512"] = dict(pivots=res.num_pivots,
                                    degenerate_pivots=int((res.pivot_log["ratio"] == 0).sum()),
                                    gpu_s=t_gpu, gpu_us_per_pivot=1e6 * t_gpu / res.num_pivots,
                                    cpu_oracle_s_1thread=t_cpu)

# C4 degenerate 2048 x 4096: 2000-pivot window, pivots/s
with dlp.Session(dlp.Problem.random(2048, 4096, 4, degenerate=True), check_interval=500) as s:
    s.run(20)
    t0 = time.perf_counter()
    st, done = s.run(2000)
    t = time.perf_counter() - t0
    r = s.result()
out["c4_degenerate_2048x4096_window"] = dict(pivots=done, s=t, pivots_per_s=done / t, status=st,
                                             degenerate_share=float((r.pivot_log["ratio"] == 0).mean()))

# C5: 4096 x (64 x 64) batch
br, t = timed(lambda: dlp.batched_solve(4096, 64, 64, 5000))
out["c5_batched_4096x64x64"] = dict(wall_s=t, kernel_ms=br.kernel_ms, lps_per_s=4096 / (br.kernel_ms / 1e3),
                                    total_pivots=int(br.num_pivots.sum()),
                                    pivots_per_s=float(br.num_pivots.sum()) / (br.kernel_ms / 1e3),
                                    all_optimal=bool((br.status == 0).all()))
# oracle on a sample of the batch (1 thread), scaled
t0 = time.perf_counter()
for k in range(64):
    A, b, c = O.gen_dense(64, 64, 5000 + k)
    O.solve_dense(A, b, c, nthreads=1, log_cap=1)
t = time.perf_counter() - t0
out["c5_batched_4096x64x64"]["cpu_oracle_lps_per_s_1thread"] = 64 / t

# f1: the reference's default instance, solved exactly
p = dlp.Problem.adalloc(1000, 1000, 1, 0.1, 0.25)
res, t_gpu = timed(lambda: dlp.solve(p))
out["f1_adalloc_1000x1000"] = dict(m=p.m, n=p.n, pivots=res.num_pivots, gpu_s=t_gpu,
                                   objective=res.objective, status=res.status,
                                   reference_mw_300_iterations_s="8.27 (BASELINE.md, 1 core, build container)",
                                   reference_mw_final_dual_value=125.37)
print(json.dumps(out, indent=1))
if a.out:
    json.dump(out, open(a.out, "w"), indent=1)
