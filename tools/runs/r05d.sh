#!/bin/bash
# r05d: tests of the ratio-workgroup knob (DLP_RATIO_THREADS) and of RCCL + lookahead on the CU split;
# c3r8 / c3r4 with 64 / 128 / 256-lane ratio workgroups (alternating); c3r8 over RCCL with lookahead
# (auto on the split) and without; then the round-5 pass lab (r05c.sh)
set -o pipefail
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ranks.py "tests/test_gpu_knobs.py::test_lookahead_chain_knobs" tests/test_gpu_knobs.py::test_ratio_threads_without_lookahead -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo FAIL tests; tail -40 $O/tests.log; exit 1; }
tail -4 $O/tests.log
run() {  # workload tag env...
timeout -k 10 300 env "${@:3}" python -u bench.py --workload $1 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1_$2.json 2> $O/$1_$2.err || { echo FAIL $1 $2; tail -20 $O/$1_$2.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 $2', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'cus', b.get('chain_cus'), 'la', b['lookahead'], 'x', d['exchange'])"
}
for w in c3r8 c3r4; do
run $w r256 DLP_RATIO_THREADS=256 && run $w r128 DLP_RATIO_THREADS=128 && run $w r64 DLP_RATIO_THREADS=64 && run $w r256b DLP_RATIO_THREADS=256 && run $w r128b DLP_RATIO_THREADS=128 && run $w r64b DLP_RATIO_THREADS=64 || exit 1
done
timeout -k 10 300 python -u bench.py --workload c3r8 --exchange rccl --no-cpu-baseline --no-eager-window --no-pivot-window > $O/c3r8_rccl_la.json 2> $O/c3r8_rccl_la.err || { echo FAIL rccl; tail -20 $O/c3r8_rccl_la.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c3r8 --exchange rccl --lookahead 0 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/c3r8_rccl_nola.json 2> $O/c3r8_rccl_nola.err || { echo FAIL rccl0; tail -20 $O/c3r8_rccl_nola.err; exit 1; }
python3 -c "
import json
for t in ('la','nola'):
    d=json.loads(open('$O/c3r8_rccl_'+t+'.json').read().strip().splitlines()[-1]); b=d['block']
    print('c3r8 rccl', t, round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'cus', b.get('chain_cus'), 'la', b['lookahead'], 'x', d['exchange'])"
bash tools/runs/r05c.sh
