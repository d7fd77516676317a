#!/usr/bin/env python3
"""Per-workgroup phases of one grouped-ring selection (slot 40 of the last block), from the
`<DLP_CHAIN_STAMPS>.wg` dump: when each workgroup started, learned q, had T0 / P[l][q], finished its
replay, its block reduce and its ticket, relative to the earliest start (us, 100 MHz clock); its CU and
wave 0's replayed steps.  Usage: python tools/wg_stamps.py <stamps.bin.wg> [nblocks]"""
import json
import sys

import numpy as np

w = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(1024, 8)
nb = int(sys.argv[2]) if len(sys.argv) > 2 else int((w[:, 0] > 0).sum())
w = w[:nb]
if nb == 0 or not (w[:, 0] > 0).all():   # no grouped-ring selection stamped this run
    print(json.dumps({"workgroups": 0}))
    sys.exit(0)
t = w[:, :6].astype(np.float64)
t0 = t[:, 0].min()
rel = (t - t0) / 100.0
ph = np.diff(rel, axis=1)
steps = w[:, 7].astype(int)
cu = w[:, 6].astype(int)
order = np.argsort(rel[:, 5])
out = {
    "workgroups": nb,
    "start_us": {"min": 0.0, "median": float(np.median(rel[:, 0])), "max": float(rel[:, 0].max())},
    "ticket_us": {"min": float(rel[:, 5].min()), "median": float(np.median(rel[:, 5])), "max": float(rel[:, 5].max())},
    "phase_median_us": dict(zip(["q", "t0", "replay", "reduce", "ticket"], [float(np.median(ph[:, k])) for k in range(5)])),
    "replay_us_by_steps": {str(s): float(np.median(ph[steps == s, 2])) for s in sorted(set(steps.tolist()))},
    "last5": [{"wg": int(i), "start": round(float(rel[i, 0]), 1), "ticket": round(float(rel[i, 5]), 1),
               "replay": round(float(ph[i, 2]), 1), "steps": int(steps[i]), "cu_hwid": hex(int(cu[i]))}
              for i in order[-5:]],
}
print(json.dumps(out, indent=1))
