#!/usr/bin/env python3
"""C5 (BASELINE.json: 4,096 independent 64 x 128 LPs, one LDS-resident workgroup each) for
profiling: `reps` batched solves; prints LPs/s and the kernel time (HIP events)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import distributedlpsolver_amd as dlp  # noqa: E402

m, n = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (64, 128)))
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dlp.batched_solve(4096, m, n, 5000, log_cap=0)   # warm
out = []
for _ in range(reps):
    t0 = time.perf_counter()
    br = dlp.batched_solve(4096, m, n, 5000, log_cap=0)
    out.append({"wall_s": time.perf_counter() - t0, "kernel_ms": br.kernel_ms,
                "pivots": int(br.num_pivots.sum()), "all_optimal": bool((br.status == 0).all())})
print(json.dumps({"m": m, "n": n, "nlp": 4096, "runs": out,
                  "lps_per_s_kernel": 4096 / (min(r["kernel_ms"] for r in out) * 1e-3)}))
