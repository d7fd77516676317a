#!/bin/bash
# r04c: drained peer push + fused select/commit (peer exchange): tests, then c3r8 block split
set -o pipefail
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_peer.py tests/test_gpu_faults.py tests/test_gpu_lookahead.py > $O/peer.log 2>&1 || { echo PEER_FAIL; grep -E "FAIL|Error|assert" $O/peer.log | head -30; tail -30 $O/peer.log; exit 1; }
tail -2 $O/peer.log
B="python -u bench.py --workload c3r8 --no-cpu-baseline --no-eager-window --no-pivot-window"
for x in peer rccl; do for la in 0 1; do
  timeout -k 10 240 $B --exchange $x --lookahead $la > $O/c3r8_${x}_la$la.json 2> $O/c3r8_${x}_la$la.err || { echo FAIL $x $la; tail -20 $O/c3r8_${x}_la$la.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/c3r8_${x}_la$la.json').read().strip().splitlines()[-1]); b=d['block']
print('$x la$la', round(d['value']), d['exchange'], 'form', d['geometry']['form'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'chain', b['chain_us_per_pivot'])"
done; done
DLP_LEAN_LCH=0 timeout -k 10 200 python -u tools/chain_stamps.py --workload c3r8 --exchange peer --lookahead 1 > $O/stamps_peer_la1.json 2>&1 || { echo STAMP_FAIL; tail -20 $O/stamps_peer_la1.json; exit 1; }
cat $O/stamps_peer_la1.json
for d in 8 16 8 16; do
DLP_RING_DEPTH=$d timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/c3_ring$d.json 2> $O/c3.err || { echo C3_FAIL; tail -20 $O/c3.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_ring$d.json').read().strip().splitlines()[-1])
print('c3 ring $d', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
done
