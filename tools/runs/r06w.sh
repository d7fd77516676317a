#!/bin/bash
# r06w: the knob suite with the new knobs (DLP_Q_U, DLP_RATIO_ROWS) against the default bits, then
# the form-23 pass with 4 rows per group (DLP_Q_U=4) against 2 at C3 and the form-23 rank geometries
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06w; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_knobs.py > $O/knobs.log 2>&1
rc=$?; tail -3 $O/knobs.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/knobs.log | head; exit $rc; }
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'form', d['geometry'].get('form'))"
}
for r in a b; do
for w in c3 c3r2 c3r4; do
run ${w}_u2_$r --workload $w || exit 1
DLP_Q_U=4 run ${w}_u4_$r --workload $w || exit 1
done
done
echo done
