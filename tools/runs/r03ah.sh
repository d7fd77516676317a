#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03ah
cd /root/repo
DLP_XMAP=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lookahead.py tests/test_gpu_defer.py -k "21" > gpurun_out/r03ah/t.log 2>&1 || { echo T_FAIL; tail -30 gpurun_out/r03ah/t.log; exit 1; }
tail -1 gpurun_out/r03ah/t.log
for x in 1 0 1 0; do
DLP_XMAP=$x timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > gpurun_out/r03ah/b.json 2> gpurun_out/r03ah/b.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03ah/b.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03ah/b.json'));print('xmap=$x', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
done
