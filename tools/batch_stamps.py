#!/usr/bin/env python3
"""Phase times of the register-resident batched kernel (C5), LP 0, first 64 pivots:
pricing (start -> barrier 1), column q + RHS to LDS (-> barrier 2), ratio test + select
(-> barrier 3), row p + pivot-row division, elimination.  Diagnostics (DLP_BATCH_STAMPS)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
path = os.path.join(ROOT, "gpurun_out", "batch_stamps.bin")
os.environ["DLP_BATCH_STAMPS"] = path
import distributedlpsolver_amd as dlp  # noqa: E402

m, n = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (64, 128)))
nlp = int(sys.argv[3]) if len(sys.argv) > 3 else 4096   # (256: one LP per CU, no co-resident LPs)
br = dlp.batched_solve(nlp, m, n, 5000, log_cap=0)
st = np.fromfile(path, dtype=np.uint64).reshape(64, 8).astype(np.float64) / 100.0   # us (100 MHz)
ok = (st[:, :6] > 0).all(axis=1)
st = st[ok]
names = ["pricing", "column q + RHS to LDS", "ratio test + select", "row p + division", "elimination"]
res = {nm: float(np.median(st[:, i + 1] - st[:, i])) for i, nm in enumerate(names)}
res["pivot total"] = float(np.median(st[:, 5] - st[:, 0]))
print(json.dumps({"m": m, "n": n, "nlp": nlp, "pivots_sampled": int(ok.sum()), "kernel_ms": br.kernel_ms,
                  "median_us": res}, indent=1))
