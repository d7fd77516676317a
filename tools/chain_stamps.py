#!/usr/bin/env python3
"""Phase times of the lookahead selection chain beside the pass.

    python tools/chain_stamps.py [bench args...]

Runs bench.py (C3 default, short) with DLP_CHAIN_STAMPS set, then reads the 64 x 16 stamps
(100 MHz wall clock) the LEAN kernels wrote for the last 64 pivots: ratio kernel workgroup 0
at start / q known / T0 and P[l][q] in / replay done / block reduce done / ticket taken, the
last workgroup at its end; the pivot-row kernel at start / step table in / replay done / end."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = os.path.join(ROOT, "gpurun_out", "chain_stamps.bin")
env = dict(os.environ, DLP_CHAIN_STAMPS=path)
cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--no-eager-window",
       "--no-pivot-window", "--steps", "3", "--warmup", "2"] + sys.argv[1:]
out = subprocess.run(cmd, env=env, check=True, capture_output=True, text=True).stdout
line = json.loads(out.strip().splitlines()[-1])
st = np.fromfile(path, dtype=np.uint64).reshape(64, 16).astype(np.float64) / 100.0   # µs
# (stamp 5, the ticket, is not taken when the ratio launch selects for the peer exchange)
fused = not (st[:, 5] > 0).any()
# (the register pivot-row kernel, used when the chain has CUs of its own, writes no stamps 8-11)
prow_stamped = (st[:, [8, 9, 10, 11]] > 0).all(axis=1).any()
ok = (st[:, [0, 1, 2, 3, 4, 6] + ([8, 9, 10, 11] if prow_stamped else []) + ([] if fused else [5])] > 0).all(axis=1)
full = st.copy()
st = st[ok]
names = ["ratio: pricing reduce (start -> q)", "ratio: T0[i][q] + P[l][q] in", "ratio: replay (lane 0)",
         "ratio: block reduce", "ratio: partials + ticket", "ratio: last workgroup select (ticket -> end)",
         "gap ratio end -> prow start", "prow: step table + T0[p] in", "prow: replay + divide",
         "prow: commit (P, objective row, pricing) / exchange push"]
pairs = [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 6), (6, 8), (8, 9), (9, 10), (10, 11)]
if fused:   # every workgroup pushes its candidate; workgroup 0 gathers them all and selects
    names = names[:4] + ["ratio: push + gather + select (wg 0: reduce -> end)"] + names[6:]
    pairs = pairs[:4] + [(4, 6)] + pairs[6:]
res = {n: float(np.median(st[:, b] - st[:, a])) for n, (a, b) in zip(names, pairs)
       if prow_stamped or (a < 8 and b < 8)}
if (st[:, 13:15] > 0).all() and not (st[:, 12] > 0).any():   # peer, fused: the commit in the prow launch
    res["prow: commit wait (push end -> chunk flag)"] = float(np.median(st[:, 13] - st[:, 11]))
    res["prow: commit (P, objective row, pricing)"] = float(np.median(st[:, 14] - st[:, 13]))
    res["pivot total (ratio start -> commit end)"] = float(np.median(st[:, 14] - st[:, 0]))
    res["pivot period (ratio start -> next ratio start)"] = float(np.median(np.diff(np.sort(st[:, 0]))))
elif (st[:, 12:15] > 0).all():   # exchange sessions: the pivot row is pushed, then committed
    for n, (a, b) in zip(["gap prow end -> commit start", "commit: wait for the row chunk",
                          "commit: P, objective row, pricing"], [(11, 12), (12, 13), (13, 14)]):
        res[n] = float(np.median(st[:, b] - st[:, a]))
    res["pivot total (ratio start -> commit end)"] = float(np.median(st[:, 14] - st[:, 0]))
    res["pivot period (ratio start -> next ratio start)"] = float(np.median(np.diff(np.sort(st[:, 0]))))
res["ratio total (start -> end)"] = float(np.median(st[:, 6] - st[:, 0]))
if prow_stamped:
    res["prow total"] = float(np.median(st[:, 11] - st[:, 8]))
res["pivot period (ratio start -> next ratio start)"] = float(np.median(np.diff(np.sort(st[:, 0]))))
# by position k in the block (slot k = pivot count mod 64): when each pivot starts after the block's
# first, and its ratio / pivot-row launch durations (-1: stamp missing)
t0 = full[0, 0]
by_slot = {"start_after_first": [round(float(full[k, 0] - t0), 1) if ok[k] else -1 for k in range(64)],
           "ratio": [round(float(full[k, 6] - full[k, 0]), 1) if ok[k] else -1 for k in range(64)],
           "prow": [round(float(full[k, 11] - full[k, 8]), 1) if ok[k] else -1 for k in range(64)]}
wg = None
if os.path.exists(path + ".wg"):   # the grouped-ring selection's per-workgroup stamps (tools/wg_stamps.py)
    wg = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "wg_stamps.py"), path + ".wg"], check=True,
                        capture_output=True, text=True).stdout
    wg = json.loads(wg) if wg.strip() and json.loads(wg)["workgroups"] > 0 else None
print(json.dumps({"pivots_sampled": int(ok.sum()), "bench_value": line["value"], "workgroups": wg,
                  "pass_ms": line["roofline"]["launch_ms"], "median_us": res, "by_slot_us": by_slot}, indent=1))
