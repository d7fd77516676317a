#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03p
cd /root/repo
for v in 4 0 4 0; do
DLP_LEAN_LCH=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --form 23 > gpurun_out/r03p/bench$v.json 2> gpurun_out/r03p/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03p/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03p/bench$v.json'));print('form 23 LCH=$v', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
done
