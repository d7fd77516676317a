#!/usr/bin/env python3
"""Where C1's end-to-end time goes: dlp.solve of the 200 x 400 LP, repeated,
and the same split into session create / run / result, for the one-launch LDS solve (auto)
and the multi-kernel path."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import distributedlpsolver_amd as dlp  # noqa: E402  (DLP_TRACE_CREATE=1: stage times on stderr)
import oracle_py as O  # noqa: E402

A, b, c = O.gen_dense(200, 400, 1)
p = dlp.Problem.dense(A, b, c)
out = {}
for mode, kw in (("lds", {}), ("multikernel", {"small_lp": -1})):
    solves = []
    for _ in range(5):
        t0 = time.perf_counter()
        r = dlp.solve(p, **kw)
        solves.append(time.perf_counter() - t0)
    parts = []
    for _ in range(3):
        t0 = time.perf_counter()
        s = dlp.Session(p, **kw)
        t1 = time.perf_counter()
        s.run(10 ** 6)
        t2 = time.perf_counter()
        res = s.result()
        t3 = time.perf_counter()
        s.close()
        t4 = time.perf_counter()
        parts.append({"create_ms": 1e3 * (t1 - t0), "run_ms": 1e3 * (t2 - t1), "result_ms": 1e3 * (t3 - t2),
                      "free_ms": 1e3 * (t4 - t3)})
    out[mode] = {"pivots": r.num_pivots, "solve_ms": [1e3 * x for x in solves], "parts": parts}
print(json.dumps(out, indent=1))
