#!/bin/bash
# r06ze: the grouped-ring pivot-row kernel (DLP_PROW_GROUP=4): knob parity, then alternating pairs
# against the register kernel at the rank geometries and C3
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06ze; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_knobs.py -k "chain_knobs or ratio_ring_rows" > $O/knobs.log 2>&1
rc=$?; tail -3 $O/knobs.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/knobs.log | head; exit $rc; }
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3))"
}
for r in a b; do
for w in c3r8 c3r4 c3r2 c3; do
run ${w}_fat_$r --workload $w || exit 1
DLP_PROW_GROUP=4 run ${w}_pg4_$r --workload $w || exit 1
done
done
echo done
