#!/bin/bash
# r05as: same-box A/B of the C5 kernel, round-5 build vs the round-4 batched kernel (dlp_batched.hip at 7d01077),
# alternating bench --workload c5
set -o pipefail
O=gpurun_out/r05as; mkdir -p $O
run() {  # tag lib
cp tools/ab/libdlp_$2.so distributedlpsolver_amd/libdlp.so || exit 1
timeout -k 10 300 python -u bench.py --workload c5 > $O/$1.json 2> $O/$1.err || { echo FAIL $1; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', round(d['value']), round(d['roofline']['frac'],3), d['roofline'].get('single_lp_us_per_pivot'))"
}
for r in a b c; do run new$r new && run prev$r c5prev || exit 1; done
cp tools/ab/libdlp_new.so distributedlpsolver_amd/libdlp.so
