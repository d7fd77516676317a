#!/bin/bash
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03h; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_defer.py -v --timeout 300 --timeout-method thread \
   -k "lds_forms" > $OUT/tests2.txt 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" $OUT/tests2.txt | tail -15
[ $rc -eq 0 ] || exit 1
bash tools/gpu_profile.sh r03h_prof || exit 1
python3 tools/pmc_summary.py gpurun_out/r03h_prof pass_d_kernel $OUT/c3_pass_pmc_traffic.json "form 21, 768-row bands, ld 65664, nt, lookahead" || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
cat $OUT/bench_default.json
