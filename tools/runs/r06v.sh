#!/bin/bash
# r06v: condensed C3 pass ceiling: the pass alone on every CU (no lookahead) against the shipped
# lookahead split; ring depth / rows per group of the form-23 pass (alternating pairs)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06v; mkdir -p $O
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'form', d['geometry'].get('form'), 'la', b.get('lookahead'))"
}
for r in a b; do
run base_$r || exit 1
run la0_$r --lookahead 0 || exit 1
run la0f21_$r --lookahead 0 --form 21 || exit 1
DLP_Q_U=4 run qu4_$r || exit 1
DLP_Q_DEPTH=6 run qd6_$r || exit 1
done
echo done
