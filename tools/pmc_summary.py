#!/usr/bin/env python3
"""Summarise a tools/gpu_profile.sh run into the committed profile files.

    python tools/pmc_summary.py <gpurun_out/tag> <kernel-substring> <out.json> [note]

Reads the FETCH_SIZE and WRITE_SIZE passes (separate rocprofv3 --pmc runs) and
the kernel-trace stats, and writes per-launch HBM traffic of the kernel:
read bytes = 2 x FETCH_SIZE KiB x 1024 (gfx950 FETCH_SIZE counts half the bytes
of a wide coalesced stream, MI355X_MICROARCH.md §HBM), write bytes = WRITE_SIZE
KiB x 1024, next to the kernel's mean duration from the trace pass."""
import csv
import glob
import json
import os
import sys


def real(vals):
    """Drop no-op launches (a deferred pass is launched as a full-block and a
    partial-block instance and exactly one of them works): < 5 % of the largest."""
    if not vals:
        return vals
    top = max(vals)
    return [v for v in vals if v >= 0.05 * top]


def counter(d, name, sub):
    vals, kname = [], None
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if sub in row.get("Kernel_Name", "") and row.get("Counter_Name") == name:
                    vals.append(float(row["Counter_Value"]))
                    kname = row["Kernel_Name"]
    return real(vals), kname


def stats(d, sub):
    """Working launches of the kernel in the kernel trace: (count, mean ns)."""
    durs = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if sub in row["Kernel_Name"]:
                    durs.append(float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))
    durs = real(durs)
    if not durs:
        return None, None
    return len(durs), sum(durs) / len(durs)


def main():
    tag, sub, out = sys.argv[1:4]
    note = sys.argv[4] if len(sys.argv) > 4 else ""
    fe, kname = counter(os.path.join(tag, "pmc_fetch"), "FETCH_SIZE", sub)
    wr, _ = counter(os.path.join(tag, "pmc_write"), "WRITE_SIZE", sub)
    calls, avg_ns = stats(os.path.join(tag, "trace"), sub)
    d = {"kernel": kname, "trace_working_launches": calls, "trace_avg_ns": avg_ns}
    # the bench line of the trace pass names the geometry (bench.py's committed_traffic key)
    try:
        with open(os.path.join(tag, "trace_bench.json")) as f:
            line = json.loads(f.read().strip().splitlines()[-1])
        d["geometry"] = line.get("geometry")
        d["trace_bench_launch_ms"] = line["roofline"]["launch_ms"]
    except (OSError, ValueError, KeyError, IndexError):
        pass
    if fe and wr:
        # the first launch after a retune / the last partial block can differ: report the mean
        rd = 2.0 * sum(fe) / len(fe) * 1024.0
        w = sum(wr) / len(wr) * 1024.0
        d.update({"FETCH_SIZE_KiB_mean": sum(fe) / len(fe), "FETCH_SIZE_launches": len(fe),
                  "WRITE_SIZE_KiB_mean": sum(wr) / len(wr), "WRITE_SIZE_launches": len(wr),
                  "hbm_read_bytes_corrected": rd, "hbm_write_bytes": w,
                  "traffic_bytes_per_launch": rd + w})
    d["note"] = note
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
