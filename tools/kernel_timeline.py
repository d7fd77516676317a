#!/usr/bin/env python3
"""Per-pivot chain timeline from a rocprofv3 kernel trace (profiles/r04p/).

    python tools/kernel_timeline.py <run_kernel_trace.csv> [blocks]

Groups the lookahead chain's launches (ratio_*, prow_*, pivot_x_*) by the pass launches
(pass_*) that bracket them and prints, for the last `blocks` full blocks, each pivot's ratio and
pivot-row durations, the gaps between them, and how far into the block the pass ended.  A
kernel trace does not perturb the kernels (the chain stamps do at the rank geometries)."""
import csv
import json
import sys

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
nblk = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows), key=lambda e: e[0])


def kind(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    for k in ("ratio_", "prow_", "pivot_x", "pass_", "seal_", "commit_", "blk_reset", "reset_cols"):
        if k in n:
            return k.rstrip("_")
    return None


ev = [(s, e, kind(n), n) for s, e, n in ev if kind(n)]
passes = [i for i, x in enumerate(ev) if x[2] == "pass"]
out = []
for bi in range(max(0, len(passes) - 1 - nblk), len(passes) - 1):
    a, b = passes[bi], passes[bi + 1]
    p0s, p0e = ev[a][0], ev[a][1]
    chain = [x for x in ev[a + 1:b] if x[2] in ("ratio", "prow", "pivot_x", "commit")]
    rat = [x for x in chain if x[2] in ("ratio", "pivot_x")]
    prw = [x for x in chain if x[2] == "prow"]
    starts = np.array([x[0] for x in rat], dtype=np.float64)
    out.append({
        "block_us": (ev[b][0] - p0s) / 1e3,
        "pass_us": (p0e - p0s) / 1e3,
        "pivots": len(rat),
        "pivots_during_pass": int(np.sum(starts < p0e)),
        "ratio_us": [round((x[1] - x[0]) / 1e3, 1) for x in rat],
        "prow_us": [round((x[1] - x[0]) / 1e3, 1) for x in prw],
        "period_us": [round(v / 1e3, 1) for v in np.diff(starts)],
        # the chain's own time: its launches summed, and how long after the pass its last launch ended
        "chain_busy_us": round(sum(x[1] - x[0] for x in chain) / 1e3, 1),
        "chain_end_after_pass_us": round((max(x[1] for x in chain) - p0e) / 1e3, 1) if chain else None,
        "reset_cols_us": [round((x[1] - x[0]) / 1e3, 1) for x in ev[a - 2:b] if x[2] == "reset_cols"][:2],
        "ratio_name": rat[0][3].replace("(anonymous namespace)::", "").split("(")[0][-60:] if rat else None,
    })
print(json.dumps(out, indent=1))
