#!/bin/bash
# r06zq: C3 form-23 pass with 4-row groups: ring depth 3 vs 2, 512-row bands (alternating)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zq; mkdir -p $O
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3))"
}
for r in a b; do
run d2_$r || exit 1
DLP_Q_DEPTH=3 run d3_$r || exit 1
run rb512_$r --rows-per-block 512 || exit 1
done
echo done
