#!/bin/bash
# r04n: per-slot chain stamps (c3r8, c3r4, C3) and the C1 graph costs
set -o pipefail
O=gpurun_out/r04n; mkdir -p $O
for w in c3r8 c3r4 c3; do
DLP_LEAN_LCH=0 timeout -k 10 200 python -u tools/chain_stamps.py --workload $w > $O/stamps_$w.json 2> $O/stamps_$w.err || { echo STAMP_FAIL $w; tail -20 $O/stamps_$w.err; exit 1; }
python3 -c "
import json
d=json.load(open('$O/stamps_$w.json')); print('$w', d['pivots_sampled'], round(d['bench_value']), {k: round(v,1) for k,v in d['median_us'].items()}); print(d['by_slot_us'])"
done
DLP_TRACE_CREATE=1 timeout -k 10 120 python -u tools/c1_overhead.py > $O/c1_overhead.json 2> $O/c1_stages.txt || { echo C1_FAIL; tail $O/c1_stages.txt; exit 1; }
tail -16 $O/c1_stages.txt
