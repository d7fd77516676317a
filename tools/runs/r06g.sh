#!/bin/bash
# r06g: condensed rank geometries (c3r8 / c3r4 / c3r2 = one rank of C3's condensed 8 / 4 / 2-GPU split):
# chain CU count A/B, and C3 with the new default (64 chain CUs)
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O
run() {  # tag workload env...
  tag=$1; w=$2; shift 2
  timeout -k 10 300 env "$@" python3 bench.py --workload $w --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'form', d['geometry']['form'], 'cus', b.get('chain_cus'), 'x', d.get('exchange'))"
}
run c3_def c3 X=0 || exit 1
for w in c3r8 c3r4 c3r2; do
run ${w}_def $w X=0 || exit 1
run ${w}_c64 $w DLP_CHAIN_CUS=64 || exit 1
run ${w}_c96 $w DLP_CHAIN_CUS=96 || exit 1
run ${w}_c128 $w DLP_CHAIN_CUS=128 || exit 1
run ${w}_c160 $w DLP_CHAIN_CUS=160 || exit 1
done
