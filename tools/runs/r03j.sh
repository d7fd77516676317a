#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03j
cd /root/repo
DLP_LEAN_LCH=0 timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lookahead.py > gpurun_out/r03j/la.log 2>&1 || { echo LA_FAIL; tail -30 gpurun_out/r03j/la.log; exit 1; }
tail -2 gpurun_out/r03j/la.log
DLP_LEAN_LCH=0 timeout -k 10 180 python -u tools/chain_stamps.py > gpurun_out/r03j/stamps0.json 2>&1 || { echo STAMP_FAIL; tail -20 gpurun_out/r03j/stamps0.json; exit 1; }
cat gpurun_out/r03j/stamps0.json
for v in 0 4 0 4; do
DLP_LEAN_LCH=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > gpurun_out/r03j/bench$v.json 2> gpurun_out/r03j/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03j/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03j/bench$v.json'));print('LCH=$v', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
done
