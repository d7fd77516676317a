#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03u
cd /root/repo
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lookahead.py -k "23" > gpurun_out/r03u/la23.log 2>&1 || { echo LA_FAIL; tail -30 gpurun_out/r03u/la23.log; exit 1; }
DLP_Q_DEPTH=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lookahead.py tests/test_gpu_defer.py -k "23" > gpurun_out/r03u/la23d2.log 2>&1 || { echo LA2_FAIL; tail -30 gpurun_out/r03u/la23d2.log; exit 1; }
tail -1 gpurun_out/r03u/la23d2.log
for cfg in "21 4" "23 2" "23 3" "21 4" "23 2" "23 3"; do set -- $cfg
DLP_Q_DEPTH=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --form $1 > gpurun_out/r03u/b.json 2> gpurun_out/r03u/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03u/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03u/b.json'));print('form $1 D $2', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
done
