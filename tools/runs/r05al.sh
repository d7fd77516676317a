#!/bin/bash
# r05al: kernel trace + stats of the C2 bench (BASELINE configs[1]): where a 22 us pivot goes
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05al; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o run -- \
    python3 $R/bench.py --workload c2 --no-cpu-baseline --no-eager-window > $O/c2_bench.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
cd $R && f=$(find $O/trace_c2 -name "*kernel_stats.csv" | head -1) && python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    print(r['Name'][:90], r['Calls'], round(float(r['AverageNs'])/1e3,2), r['Percentage'])" | head -12
