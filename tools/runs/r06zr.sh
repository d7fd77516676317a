#!/bin/bash
# r06zr: C3 band height with 4-row pass groups (alternating triples), and c3r2
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zr; mkdir -p $O
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'rb', d['geometry']['rows_per_block'])"
}
for r in a b c; do
run rb768_$r || exit 1
run rb512_$r --rows-per-block 512 || exit 1
run rb640_$r --rows-per-block 640 || exit 1
run rb384_$r --rows-per-block 384 || exit 1
done
for r in a b; do
run c3r2_768_$r --workload c3r2 || exit 1
run c3r2_512_$r --workload c3r2 --rows-per-block 512 || exit 1
done
echo done
