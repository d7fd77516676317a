#!/usr/bin/env python3
"""Per-launch means of rocprofv3 SQ counters for one kernel (tools/sq_counters.sh):

    python tools/sq_summary.py <pmc dir> <kernel-substring>

Launches doing no work (a deferred pass is launched as a full-block and a
partial-block instance, exactly one of which works) are dropped: SQ_WAVE_CYCLES
(else SQ_INSTS_VALU, else SQ_WAVES) under 5 % of the largest.  Fractions are of SQ_WAVE_CYCLES (quad-cycles; the
three SQ states WAIT_ANY, WAIT_INST_ANY and ACTIVE_INST_ANY are disjoint:
MI355X_MICROARCH.md §rocprofv3 PMC slots)."""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d, sub = sys.argv[1], sys.argv[2]
    per = collections.defaultdict(dict)   # dispatch id -> counter -> value
    name = None
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if sub not in row.get("Kernel_Name", ""):
                    continue
                name = row["Kernel_Name"]
                key = (path, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                per[key][row["Counter_Name"]] = per[key].get(row["Counter_Name"], 0.0) + \
                    float(row["Counter_Value"])
    ref = next((k for k in ("SQ_WAVE_CYCLES", "SQ_INSTS_VALU", "SQ_WAVES", "SQ_BUSY_CYCLES")
                if any(k in v for v in per.values())), None) or \
        next(iter(sorted({k for v in per.values() for k in v})), None)
    launches = [v for v in per.values() if ref in v]
    if not launches:
        raise SystemExit(f"no launches of {sub!r} under {d}")
    top = max(v[ref] for v in launches)
    launches = [v for v in launches if v[ref] >= 0.05 * top]
    keys = sorted({k for v in launches for k in v})
    out = {"kernel": name, "launches": len(launches)}
    for k in keys:
        out[k] = sum(v.get(k, 0.0) for v in launches) / len(launches)
    wc = out.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
            if k in out:
                out["frac_" + k[3:].lower()] = out[k] / wc
        if out.get("SQ_WAVES"):
            out["wave_cycles_per_wave"] = wc / out["SQ_WAVES"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
