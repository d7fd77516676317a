#!/bin/bash
# r04ak: the chain's ratio kernel with two ring pairs per wait on its own CUs (DLP_WIDE_RATIO A/B)
set -o pipefail
O=gpurun_out/r04ak; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_knobs.py -m gpu > $O/tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # workload tag env...
timeout -k 10 300 env "${@:3}" python -u bench.py --workload $1 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1_$2.json 2> $O/$1.err || { echo FAIL $1 $2; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 $2', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'cus', b.get('chain_cus'))"
}
for w in c3r8 c3r4 c3r2; do
run $w wide DLP_WIDE_RATIO=1 && run $w ring DLP_WIDE_RATIO=0 && run $w wide2 DLP_WIDE_RATIO=1 && run $w ring2 DLP_WIDE_RATIO=0 || exit 1
done
