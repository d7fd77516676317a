#!/bin/bash
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03e; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1; rc=$?
grep -E "passed|failed|FAILED|ERROR" $OUT/gpu_tests.txt | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for f in 21 23; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-eager-window --lookahead 0 --form $f > $OUT/bench_nola_f$f.json 2>> $OUT/bench.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/bench_nola_f$f.json').read().strip().splitlines()[-1]); print('no-lookahead form', $f, round(d['value']), 'pass ms', round(d['roofline']['launch_ms'],3), 'frac', round(d['roofline']['frac'],3), d['pivot_log_vs_oracle']['bit_identical'])"
done
timeout -k 10 90 python3 tools/c1_overhead.py > $OUT/c1_overhead.json 2> $OUT/c1_overhead.err || exit 1
bash tools/c5_profile.sh r03e_c5 || exit 1
