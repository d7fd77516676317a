#!/bin/bash
# r06a: round-6 changes on the GPU: co-located rank processes with disjoint chain CU slices from the exchange
# records (no test knob), C4 2048 x 4096 degenerate digests, the cached batch context (C5 wall rate)
set -o pipefail
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -x -v -k "c4 or c5" --timeout 240 --timeout-method thread > $O/large.log 2>&1 || { echo FAIL large; tail -40 $O/large.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/large.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_knobs.py -x -v -k "batch" --timeout 120 --timeout-method thread > $O/batch.log 2>&1 || { echo FAIL batch; tail -40 $O/batch.log; exit 1; }
grep -E "passed|failed" $O/batch.log
timeout -k 10 200 python -u bench.py --workload c5 --cpu-seconds 2 > $O/bench_c5.json 2> $O/bench_c5.err || { echo FAIL c5; tail -20 $O/bench_c5.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c5.json').read().strip().splitlines()[-1])
print('c5 kernel', round(d['value']), 'wall', round(d['wall_lps_per_s']), 'ratio', round(d['wall_lps_per_s']/d['value'],3))"
timeout -k 10 900 python -u -m pytest tests/test_gpu_ranks.py -x -v --timeout 420 --timeout-method thread > $O/ranks.log 2>&1 || { echo FAIL ranks; tail -60 $O/ranks.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/ranks.log
