#!/bin/bash
# r06m: condensed C3, chain on 64 CUs: form-23 ring depth on the pass's own 192 CUs (DLP_Q_DEPTH), alternating
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06m; mkdir -p $O
run() {  # tag env...
  tag=$1; shift
  timeout -k 10 300 env "$@" python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3))"
}
for r in a b; do
run d4_$r X=0 || exit 1
run d6_$r DLP_Q_DEPTH=6 || exit 1
run d8_$r DLP_Q_DEPTH=8 || exit 1
run d3_$r DLP_Q_DEPTH=3 || exit 1
done
