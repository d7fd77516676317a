#!/bin/bash
# r04h: lookahead auto at K = 64 streaming (peer ranks too); tests; rank geometries; C1 untraced
set -o pipefail
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_peer.py tests/test_gpu_lookahead.py tests/test_gpu_c3_rowblock.py > $O/tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in c3r8 c3r4 c3r2; do
timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-eager-window --no-pivot-window > $O/${w}_auto.json 2> $O/$w.err || { echo FAIL $w; tail -20 $O/$w.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/${w}_auto.json').read().strip().splitlines()[-1]); b=d['block']
print('$w auto', round(d['value']), d['exchange'], 'la', b['lookahead'], 'form', d['geometry']['form'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3))"
done
timeout -k 10 120 python -u tools/c1_overhead.py > $O/c1_overhead.json 2> $O/c1.err || { echo C1_FAIL; tail $O/c1.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/c1_overhead.json'))
for k,v in d.items(): print('c1', k, v['pivots'], [round(x,2) for x in v['solve_ms']], {a: round(b,3) for a,b in v['parts'][-1].items()})"
