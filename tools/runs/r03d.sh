#!/bin/bash
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03d; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_lookahead.py tests/test_gpu_peer.py tests/test_gpu_c3_rowblock.py tests/test_gpu_large.py -v --timeout 300 --timeout-method thread \
   -k "form21 or lookahead_k64 or lookahead_rccl or step_api_multi_rank or c3_full_blocks or peer or c3_row_partition or bench_window" > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" $OUT/tests.txt | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for f in 21 23 21 23; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-eager-window --form $f > $OUT/bench_f$f.json 2>> $OUT/bench.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/bench_f$f.json').read().strip().splitlines()[-1]); print('form', $f, round(d['value']), 'pass ms', round(d['roofline']['launch_ms'],3), 'frac', round(d['roofline']['frac'],3), d['pivot_log_vs_oracle'])"
done
