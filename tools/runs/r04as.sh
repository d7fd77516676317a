#!/bin/bash
# r04as: the register pivot-row kernel's rows in flight (DLP_PROW_CH = 16 / 24 / 32) on the CU split
set -o pipefail
O=gpurun_out/r04as; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_knobs.py -m gpu -k "chain or split" > $O/tests.log 2>&1 || { echo TEST_FAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # workload tag env...
timeout -k 10 300 env "${@:3}" python -u bench.py --workload $1 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1_$2.json 2> $O/$1.err || { echo FAIL $1 $2; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 $2', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'cus', b.get('chain_cus'))"
}
for w in c3r8 c3r4; do
run $w ch16 DLP_PROW_CH=16 && run $w ch24 DLP_PROW_CH=24 && run $w ch32 DLP_PROW_CH=32 && run $w ch16b DLP_PROW_CH=16 && run $w ch32b DLP_PROW_CH=32 || exit 1
done
