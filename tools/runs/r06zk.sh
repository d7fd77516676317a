#!/bin/bash
# r06zk: ratio workgroup shape at the rank geometries with the retuned chain budget (alternating pairs)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zk; mkdir -p $O
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'chain_cus', b['chain_cus'])"
}
for r in a b; do
for w in c3r8 c3r4; do
run ${w}_def_$r --workload $w || exit 1
DLP_RATIO_ROWS=32 run ${w}_rows32_$r --workload $w || exit 1
DLP_RATIO_THREADS=256 run ${w}_t256_$r --workload $w || exit 1
done
DLP_RATIO_ROWS=0 run c3r2_lean_$r --workload c3r2 || exit 1
run c3r2_def_$r --workload c3r2 || exit 1
done
echo done
