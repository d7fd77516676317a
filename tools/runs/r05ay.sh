#!/bin/bash
# r05ay: C5 with wave 0's RHS division issued beside the pivot-row division (uniform result kept in SGPRs);
# the batched tests, then a same-box A/B against r05at
set -o pipefail
O=gpurun_out/r05ay; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py::test_c5_full_batch tests/test_gpu_parity.py -k "batched or c5" tests/test_gpu_knobs.py::test_batched_lds_kernel_knob -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo FAIL tests; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # tag lib
cp tools/ab/libdlp_$2.so distributedlpsolver_amd/libdlp.so || exit 1
timeout -k 10 300 python -u bench.py --workload c5 > $O/$1.json 2> $O/$1.err || { echo FAIL $1; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', round(d['value']), round(d['roofline']['frac'],3), round(d['roofline'].get('single_lp_us_per_pivot'),3))"
}
for r in a b c; do run new$r new && run prev$r c5prev || exit 1; done
cp tools/ab/libdlp_new.so distributedlpsolver_amd/libdlp.so
