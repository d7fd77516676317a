#!/usr/bin/env python3
"""Secondary measurements (not the bench.py headline): full solves of the
small / degenerate configs, the C5 batch, and the reference's own generated
instance, each next to the CPU oracle (same pivot rule) on this host.

    python tools/bench_extra.py [--out FILE] [--threads 16]

Rows (BASELINE.json configs):
  C1   200 x 400 dense, seed 1, solved to optimality
  C4   degenerate 256 x 512 (seed 4), 2048 x 4096 pivot window
  C5   4096 independent 64 x 64 and 64 x 128 LPs, one LDS-resident workgroup each
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

def small_solve(A, b, c, key, **extra):
    """Full solve three ways: dlp_solve end to end (auto = the one-launch LDS
    solve for a tableau this small), the same with small_lp = -1 (the
    multi-kernel path), and the device time per pivot of the LDS solve (HIP
    events around its launches, one window)."""
    p = dlp.Problem.dense(A, b, c)
    res, t_gpu = timed(lambda: dlp.solve(p))
    res_mk, t_mk = timed(lambda: dlp.solve(p, small_lp=-1))
    with dlp.Session(p, small_lp=1, timing=1, check_interval=10 ** 6) as s:
        s.run(10 ** 6)
        _, dev_ms, _ = s.update_stats()
        npiv = s.result().num_pivots
    ref, t_cpu = timed(lambda: O.solve_dense(A, b, c, nthreads=1))
    for r in (res, res_mk):
        assert np.ascontiguousarray(r.pivot_log).tobytes() == np.ascontiguousarray(ref.pivot_log).tobytes()
    out[key] = dict(pivots=res.num_pivots, gpu_s=t_gpu, gpu_us_per_pivot=1e6 * t_gpu / res.num_pivots,
                    lds_solve_device_us_per_pivot=1e3 * dev_ms / npiv,
                    multikernel_gpu_s=t_mk, multikernel_us_per_pivot=1e6 * t_mk / res_mk.num_pivots,
                    cpu_oracle_s_1thread=t_cpu, objective=res.objective, **extra)
    return res


# C1: full solve (host-supplied data), GPU vs oracle
A, b, c = O.gen_dense(200, 400, 1)
small_solve(A, b, c, "c1_full_solve")

# C4 degenerate 256 x 512 full solve
A, b, c = O.gen_dense(256, 512, 4, degenerate=True)
r = small_solve(A, b, c, "c4_degenerate_256x512")
out["c4_degenerate_256x512"]["degenerate_pivots"] = int((r.pivot_log["ratio"] == 0).sum())

# C4 degenerate 2048 x 4096: 2000-pivot window, pivots/s
with dlp.Session(dlp.Problem.random(2048, 4096, 4, degenerate=True), check_interval=500) as s:
    s.run(20)
    t0 = time.perf_counter()
    st, done = s.run(2000)
    t = time.perf_counter() - t0
    r = s.result()
out["c4_degenerate_2048x4096_window"] = dict(pivots=done, s=t, pivots_per_s=done / t, status=st,
                                             degenerate_share=float((r.pivot_log["ratio"] == 0).mean()))

# C5: 4096 x (64 x 64) and 4096 x (64 x 128) (BASELINE.json's shape) batches
for (cm, cn) in ((64, 64), (64, 128)):
    br, t = timed(lambda: dlp.batched_solve(4096, cm, cn, 5000))
    key = f"c5_batched_4096x{cm}x{cn}"
    tp = int(br.num_pivots.sum())
    # LDS bytes per pivot of one LP: the elimination reads and writes the (m+1) x (N+1)
    # tableau once (16 B per element), plus a 1-D read of the pivot row and column
    lds_bytes = tp * (16.0 * (cm + 1) * (cm + cn + 1))
    out[key] = dict(wall_s=t, kernel_ms=br.kernel_ms, lps_per_s=4096 / (br.kernel_ms / 1e3),
                    total_pivots=tp, pivots_per_s=tp / (br.kernel_ms / 1e3),
                    all_optimal=bool((br.status == 0).all()),
                    lds_elimination_tbs=lds_bytes / (br.kernel_ms / 1e3) / 1e12)
    # oracle on a sample of the batch (1 thread), scaled
    t0 = time.perf_counter()
    for k in range(64):
        A, b, c = O.gen_dense(cm, cn, 5000 + k)
        O.solve_dense(A, b, c, nthreads=1, log_cap=1)
    t = time.perf_counter() - t0
    out[key]["cpu_oracle_lps_per_s_1thread"] = 64 / t

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
