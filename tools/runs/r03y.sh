#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03y
cd /root/repo
DLP_LDS_PART=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lookahead.py > gpurun_out/r03y/la.log 2>&1 || { echo LA_FAIL; tail -30 gpurun_out/r03y/la.log; exit 1; }
tail -1 gpurun_out/r03y/la.log
for cfg in "21 0" "23 1" "21 1" "23 0" "21 0" "23 1" "21 1"; do set -- $cfg
DLP_LDS_PART=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --form $1 > gpurun_out/r03y/b.json 2> gpurun_out/r03y/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03y/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03y/b.json'));print('form $1 part $2', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
done
