#!/bin/bash
# r05aq: the chain kernels read the state's fields (status, block, pivots) in one round trip ahead of the status branch:
# the deferred, lookahead, peer and large-tableau tests, then C2 / C3 / c3r8 benches
set -o pipefail
O=gpurun_out/r05aq; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_lookahead.py tests/test_gpu_peer.py tests/test_gpu_large.py tests/test_gpu_parity.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo FAIL tests; grep -E "Error|assert" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # tag args
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window $2 > $O/$1.json 2> $O/$1.err || { echo FAIL $1; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', round(d['value']))"
}
for r in a b; do run c2$r "--workload c2" && run c3$r "" && run c3r8$r "--workload c3r8" || exit 1; done
