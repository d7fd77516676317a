#!/bin/bash
# r05an: C5 as r05ak plus the ratio test in the wave that holds the entering column (no second barrier; RHS copies in every wave);
# the batched tests (every LP of both C5 batches against the oracle's digests), stamps, the c5 bench line
set -o pipefail
O=gpurun_out/r05an; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py::test_c5_full_batch tests/test_gpu_parity.py -k "batched or c5" tests/test_gpu_knobs.py::test_batched_lds_kernel_knob -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo FAIL tests; grep -E "Error|assert" $O/tests.log | head; tail -5 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log
for a in "64 128 4096" "64 128 256" "64 64 4096"; do
t=$(echo $a | tr ' ' _)
timeout -k 10 120 python -u tools/batch_stamps.py $a > $O/stamps_$t.json 2> $O/stamps_$t.err || { echo FAIL $t; tail -5 $O/stamps_$t.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/stamps_$t.json')); print('$t', round(d['kernel_ms'],3), {k: round(v,2) for k,v in d['median_us'].items()})"
done
for r in a b; do
timeout -k 10 300 python -u bench.py --workload c5 > $O/c5_$r.json 2> $O/c5_$r.err || { echo FAIL c5; tail -10 $O/c5_$r.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/c5_$r.json').read().strip().splitlines()[-1]); print('c5', round(d['value']), d['roofline']['frac'])"
done
