#!/bin/bash
# r04e: fused peer chain on 1-rank exchange sessions too; C5 DPP shipped
set -o pipefail
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_peer.py tests/test_gpu_faults.py tests/test_gpu_lookahead.py > $O/peer.log 2>&1 || { echo PEER_FAIL; grep -E "FAIL|Error|assert" $O/peer.log | head -30; tail -30 $O/peer.log; exit 1; }
tail -1 $O/peer.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_large.py tests/test_gpu_parity.py -k "c5 or batched" > $O/c5.log 2>&1 || { echo C5_FAIL; tail -30 $O/c5.log; exit 1; }
tail -1 $O/c5.log
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
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_la0 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c3r8 --exchange peer --lookahead 0 --no-cpu-baseline --no-eager-window --no-pivot-window > $GRAFT_REPO_ROOT/$O/prof_la0.json 2> $GRAFT_REPO_ROOT/$O/prof_la0.err || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/$O/prof_la0.err; exit 1; }
echo r04e done
