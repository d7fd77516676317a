#!/bin/bash
# r04aj: the split policy v2 (form 23 on the split above 4,096 rows; 128 / 64 chain CUs): tests + benches
set -o pipefail
O=gpurun_out/r04aj; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_knobs.py tests/test_gpu_peer.py tests/test_gpu_lookahead.py tests/test_gpu_c3_rowblock.py tests/test_gpu_large.py -m gpu > $O/tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in c3r8 c3r4 c3r2 c3; do for r in 1 2; do
timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-eager-window --no-pivot-window > $O/${w}_$r.json 2> $O/$w.err || { echo FAIL $w; tail -20 $O/$w.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/${w}_$r.json').read().strip().splitlines()[-1]); b=d['block']
print('$w', round(d['value']), 'form', d['geometry']['form'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'cus', b.get('chain_cus'), 'bit', (d.get('pivot_log_vs_oracle') or {}).get('bit_identical'))"
done; done
