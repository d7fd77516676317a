#!/bin/bash
# r06l: condensed C3 with the chain on 64 CUs: pass form 21 / 22 (MFMA) / 23 (default) on the other 192, alternating
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06l; mkdir -p $O
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'form', d['geometry']['form'], 'cus', b.get('chain_cus'))"
}
for r in a b; do
run f23_$r || exit 1
run f21_$r --form 21 || exit 1
run f22_$r --form 22 || exit 1
done
