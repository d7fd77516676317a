#!/bin/bash
# r06u: condensed C3 on the shipped build: pass band height (rows per band), pass form, and the chain's
# CU count now that the selection runs the grouped ring (alternating pairs)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06u; mkdir -p $O
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'rb', d['geometry']['rows_per_block'], 'form', d['geometry'].get('form'))"
}
for r in a b; do
run base_$r || exit 1
run rb512_$r --rows-per-block 512 || exit 1
run rb1024_$r --rows-per-block 1024 || exit 1
DLP_CHAIN_CUS=32 run cus32_$r || exit 1
DLP_CHAIN_CUS=96 run cus96_$r || exit 1
run form21_$r --form 21 || exit 1
done
echo done
