#!/bin/bash
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03g; mkdir -p $OUT
DLP_TRACE_CREATE=1 timeout -k 10 90 python3 tools/c1_overhead.py > $OUT/c1_overhead.json 2> $OUT/c1_stages.txt || exit 1
python3 -c "
import json; d=json.load(open('$OUT/c1_overhead.json'))
for k,v in d.items(): print(k, [round(x,2) for x in v['solve_ms']], [{a:round(b,3) for a,b in p.items()} for p in v['parts']][-1])"
for a in "" "--ld-align 128" "--rows-per-block 1024" "--ld-align 128 --rows-per-block 1024" "" "--ld-align 128" "--rows-per-block 1536" "--ld-align 128 --rows-per-block 1536"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-eager-window $a > $OUT/b.json 2>> $OUT/bench.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('[$a]', round(d['value']), 'pass ms', round(d['roofline']['launch_ms'],3), 'frac', round(d['roofline']['frac'],3), 'ld', d['config']['ld'], 'rb', d['geometry']['rows_per_block'], d['pivot_log_vs_oracle']['bit_identical'])"
done
