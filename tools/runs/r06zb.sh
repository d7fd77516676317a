#!/bin/bash
# r06zb: condensed C3 row stride (ld) sweep: the pass alone (no lookahead) and in situ
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zb; mkdir -p $O
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'ld', d['geometry'].get('ld'))"
}
for a in 16 64 128 256 512 1024 2048; do
run la_$a --ld-align $a || exit 1
run la0_$a --ld-align $a --lookahead 0 || exit 1
done
echo done
