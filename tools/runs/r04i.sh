#!/bin/bash
# r04i: the peer pivot in ONE launch (selection record to the pivot-row workgroups): tests, A/B
set -o pipefail
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_peer.py tests/test_gpu_faults.py tests/test_gpu_lookahead.py > $O/tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for w in c3r8 c3r4 c3r2; do for one in 1 0; do
DLP_PEER_ONELAUNCH=$one timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-eager-window --no-pivot-window > $O/${w}_one$one.json 2> $O/$w.err || { echo FAIL $w $one; tail -20 $O/$w.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/${w}_one$one.json').read().strip().splitlines()[-1]); b=d['block']
print('$w onelaunch $one', round(d['value']), d['exchange'], 'la', b['lookahead'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3))"
done; done
for la in 0 1; do
timeout -k 10 300 python -u bench.py --workload c3r8 --lookahead $la --no-cpu-baseline --no-eager-window --no-pivot-window > $O/c3r8_la$la.json 2> $O/c3r8.err || { echo FAIL c3r8 $la; tail -20 $O/c3r8.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3r8_la$la.json').read().strip().splitlines()[-1]); b=d['block']
print('c3r8 onelaunch la$la', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'chain', b['chain_us_per_pivot'])"
done
DLP_LEAN_LCH=0 timeout -k 10 200 python -u tools/chain_stamps.py --workload c3r8 > $O/stamps_c3r8.json 2>&1 || { echo STAMP_FAIL; tail -20 $O/stamps_c3r8.json; exit 1; }
python3 -c "
import json
d=json.load(open('$O/stamps_c3r8.json')); print('stamps c3r8', d['pivots_sampled'], round(d['bench_value']), {k: round(v,1) for k,v in d['median_us'].items()})"
