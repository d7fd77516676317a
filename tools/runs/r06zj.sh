#!/bin/bash
# r06zj: the new chain CU policy (condensed rank alone on its device: 96 CUs up to 8,192 rows, 128 at
# 16,384): the lookahead / knob / rank / large suites against the oracle, then the rank geometries' bench lines
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zj; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_knobs.py tests/test_gpu_ranks.py tests/test_gpu_lookahead.py tests/test_gpu_large.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/tests.log | head; exit $rc; }
for w in c3r8 c3r4 c3r2 c3; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --workload $w > $O/$w.json 2> $O/$w.err || { echo FAIL $w; tail -20 $O/$w.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$w.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$w', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'chain_cus', b['chain_cus'], 'form', d['geometry'].get('form'))"
done
echo done
