#!/bin/bash
# r05aa: L2 hit rate of the chain kernels at c3r8 and C3 (PMC TCC_HIT_sum / TCC_MISS_sum per dispatch; the profiler
# serialises dispatches, so the pass is not beside the chain here) and FETCH_SIZE at c3r8
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05aa; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/c3r8_hit -o run -- \
    python3 $R/bench.py --workload c3r8 --no-cpu-baseline --no-eager-window --no-pivot-window --steps 3 --warmup 2 > $O/c3r8_hit.json 2> $O/c3r8_hit.err || { tail -20 $O/c3r8_hit.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c3r8_fetch -o run -- \
    python3 $R/bench.py --workload c3r8 --no-cpu-baseline --no-eager-window --no-pivot-window --steps 3 --warmup 2 > $O/c3r8_fetch.json 2> $O/c3r8_fetch.err || { tail -20 $O/c3r8_fetch.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/c3_hit -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --steps 3 --warmup 2 > $O/c3_hit.json 2> $O/c3_hit.err || { tail -20 $O/c3_hit.err; exit 1; }
cd $R && python3 - <<'PY'
import csv, collections, re, glob
for tag in ("c3r8_hit", "c3r8_fetch", "c3_hit"):
    f = glob.glob(f"gpurun_out/r05aa/{tag}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]; m = re.search(r"(\w+_kernel(<[^(]*>)?)", n); k = m.group(1) if m else n[:40]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(tag)
    for k, d in agg.items():
        med = {c: sorted(v)[len(v)//2] for c, v in d.items()}
        n = len(next(iter(d.values())))
        if "TCC_HIT_sum" in med:
            h, mi = med["TCC_HIT_sum"], med["TCC_MISS_sum"]
            print(f"  {k[:60]:60s} n={n:4d} hit={h:10.0f} miss={mi:10.0f} hit_rate={h/max(h+mi,1):.3f}")
        else:
            print(f"  {k[:60]:60s} n={n:4d} " + " ".join(f"{c}={v:.1f}" for c, v in med.items()))
PY
