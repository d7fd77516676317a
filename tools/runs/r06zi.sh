#!/bin/bash
# r06zi: chain CU count at the condensed rank geometries, second sweep
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zi; mkdir -p $O
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'chain_cus', b['chain_cus'], 'form', d['geometry'].get('form'))"
}
for r in a b; do
DLP_CHAIN_CUS=64 run c3r8_64_$r --workload c3r8 || exit 1
DLP_CHAIN_CUS=96 run c3r8_96_$r --workload c3r8 || exit 1
DLP_CHAIN_CUS=64 run c3r4_64_$r --workload c3r4 || exit 1
DLP_CHAIN_CUS=96 run c3r4_96_$r --workload c3r4 || exit 1
DLP_CHAIN_CUS=128 run c3r2_128_$r --workload c3r2 || exit 1
DLP_CHAIN_CUS=160 run c3r2_160_$r --workload c3r2 || exit 1
done
echo done
