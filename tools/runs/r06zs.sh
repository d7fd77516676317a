#!/bin/bash
# r06zs: the one-launch peer pivot on the condensed tableau with the chain on its own CUs (pivot_x_ring_kernel,
# DLP_PEER_ONELAUNCH=1): parity (peer suite; the rank-process suite with it on), then alternating pairs
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zs; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_peer.py > $O/peer.log 2>&1
rc=$?; tail -2 $O/peer.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/peer.log | head; exit $rc; }
DLP_PEER_ONELAUNCH=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 420 --timeout-method thread -m gpu tests/test_gpu_ranks.py > $O/ranks_onelaunch.log 2>&1
rc=$?; tail -2 $O/ranks_onelaunch.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/ranks_onelaunch.log | head; exit $rc; }
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'chain_cus', b['chain_cus'])"
}
for r in a b; do
for w in c3r8 c3r4 c3r2; do
run ${w}_two_$r --workload $w || exit 1
DLP_PEER_ONELAUNCH=1 run ${w}_one_$r --workload $w || exit 1
done
done
echo done
