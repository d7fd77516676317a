#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03w
cd /root/repo
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_defer.py tests/test_gpu_lookahead.py -k "24" > gpurun_out/r03w/t24.log 2>&1 || { echo T24_FAIL; tail -30 gpurun_out/r03w/t24.log; exit 1; }
tail -2 gpurun_out/r03w/t24.log
for cfg in "21 4" "24 4" "24 3" "24 5" "21 4" "24 4" "24 3" "24 5"; do set -- $cfg
DLP_E_DEPTH=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --form $1 > gpurun_out/r03w/b.json 2> gpurun_out/r03w/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03w/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03w/b.json'));print('form $1 D $2', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
done
for cfg in "21" "24"; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --lookahead 0 --form $cfg > gpurun_out/r03w/b.json 2> gpurun_out/r03w/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03w/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03w/b.json'));print('no-lookahead form $cfg', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
done
