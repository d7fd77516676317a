#!/bin/bash
# r05az: rocprofv3 kernel trace + stats of the c5 bench line on the final build (the C5 line reproduced
# from a profile)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05az; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o run -- \
    python3 $R/bench.py --workload c5 > $O/c5_bench.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
cd $R && f=$(find $O/trace_c5 -name "*kernel_stats.csv" | head -1) && python3 -c "
import csv, json
for r in csv.DictReader(open('$f')):
    print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3,2))
d=json.loads(open('$O/c5_bench.json').read().strip().splitlines()[-1]); print('bench', round(d['value']), d.get('ms_per_step'), json.dumps(d['roofline'])[:300])" | head -12
