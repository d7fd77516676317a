#!/bin/bash
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03f; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_lookahead.py tests/test_gpu_peer.py tests/test_gpu_large.py tests/test_gpu_parity.py -v --timeout 300 --timeout-method thread \
   -k "form21 or lookahead_k64 or lookahead_rccl or step_api_multi_rank or c3_full_blocks or peer_exchange_dense or sparse or adalloc or degenerate" > $OUT/tests.txt 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" $OUT/tests.txt | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for a in "--form 21" "--lookahead 0 --form 23" "--form 21" "--lookahead 0 --form 23"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-eager-window $a > $OUT/b.json 2>> $OUT/bench.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); print('$a', round(d['value']), 'pass ms', round(d['roofline']['launch_ms'],3), 'frac', round(d['roofline']['frac'],3), d['pivot_log_vs_oracle']['bit_identical'])"
done
bash tools/_lab6.sh
DLP_TRACE_CREATE=1 timeout -k 10 90 python3 tools/c1_overhead.py > gpurun_out/r03f/c1_overhead.json 2> gpurun_out/r03f/c1_stages.txt || exit 1
tail -24 gpurun_out/r03f/c1_stages.txt
