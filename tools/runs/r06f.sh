#!/bin/bash
# r06f: condensed C3 — chain/pass CU split A/B (the pass is now shorter than the chain), alternating
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O
run() {  # tag env...
  tag=$1; shift
  timeout -k 10 300 env "$@" python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'form', d['geometry']['form'], 'cus', b.get('chain_cus'))"
}
for r in a b; do
run def_$r X=0 || exit 1
run c32_$r DLP_CHAIN_CUS=32 || exit 1
run c64_$r DLP_CHAIN_CUS=64 || exit 1
run c96_$r DLP_CHAIN_CUS=96 || exit 1
done
