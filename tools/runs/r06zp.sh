#!/bin/bash
# r06zp: form-23 pass with its DMA row offsets as scalars (no per-lane 64-bit multiplies): parity, then
# alternating pairs against the previous library (abtree/, the same bench.py)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zp; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_large.py tests/test_gpu_defer.py \
    tests/test_gpu_knobs.py -k "not cluster and not batched" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/tests.log | head; exit $rc; }
run() {  # tag dir args...
  tag=$1; dir=$2; shift 2
  (cd $dir && timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@") > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3))"
}
for r in a b; do
for w in c3 c3r2 c3r4; do
run ${w}_new_$r $R --workload $w || exit 1
run ${w}_old_$r $R/abtree --workload $w || exit 1
done
run c3la0_new_$r $R --lookahead 0 || exit 1
run c3la0_old_$r $R/abtree --lookahead 0 || exit 1
done
echo done
