#!/bin/bash
# r05r: C3 with the chain's LDS rings 16 deep (DLP_CHAIN_RING=16: 16 ring DMAs in flight per wave in the
# ratio and pivot-row launches instead of 8) beside the form-21, form-23 and form-22 (LEAN chain) passes;
# alternating.  The r05p stamps put the ratio launch's time in the straggler's sealed replay.
set -o pipefail
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 600 python -u -m pytest "tests/test_gpu_knobs.py::test_lookahead_chain_knobs" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo FAIL tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # tag args env...
timeout -k 10 300 env "${@:3}" python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window $2 > $O/c3_$1.json 2> $O/c3_$1.err || { echo FAIL $1; tail -20 $O/c3_$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'form', d['geometry']['form'])"
}
for r in a b; do
run def$r "" X=0 && run r16$r "" DLP_CHAIN_RING=16 && run f23$r "--form 23" X=0 && run f23r16$r "--form 23" DLP_CHAIN_RING=16 \
 && run f22l$r "--form 22" DLP_MID_CHAIN=0 && run f22lr16$r "--form 22" DLP_MID_CHAIN=0 DLP_CHAIN_RING=16 || exit 1
done
timeout -k 10 300 env DLP_CHAIN_RING=16 python -u tools/chain_stamps.py > $O/stamps_r16.json 2> $O/stamps_r16.err || { echo FAIL stamps; tail -20 $O/stamps_r16.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/stamps_r16.json')); print(d['bench_value'], {k: round(v,1) for k,v in d['median_us'].items()})"
