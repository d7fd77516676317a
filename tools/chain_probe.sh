#!/bin/bash
# Bench + kernel-trace stats of the C3 default (run through gpurun): tools/chain_probe.sh <tag> [bench args]
set -o pipefail
R=$(pwd); TAG=$1; shift
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > $OUT/b.json || exit 1
python3 -c "
import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('bench', round(d['value']), round(d['roofline']['launch_ms'],3), d['config']['lookahead'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $R/bench.py --no-cpu-baseline --no-pivot-window --steps 6 --warmup 2 "$@" > /dev/null 2>&1 || exit 1
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/prof/run_kernel_stats.csv')))[:5]: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3, 1))"
