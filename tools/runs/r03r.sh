#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03r
cd /root/repo
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lookahead.py > gpurun_out/r03r/la.log 2>&1 || { echo LA_FAIL; tail -30 gpurun_out/r03r/la.log; exit 1; }
tail -2 gpurun_out/r03r/la.log
timeout -k 10 180 python -u tools/chain_stamps.py > gpurun_out/r03r/stamps.json 2>&1 || { echo STAMP_FAIL; tail -20 gpurun_out/r03r/stamps.json; exit 1; }
cat gpurun_out/r03r/stamps.json
for v in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > gpurun_out/r03r/bench$v.json 2> gpurun_out/r03r/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03r/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03r/bench$v.json'));print('run $v', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
done
