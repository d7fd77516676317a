#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03af
cd /root/repo
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_defer.py tests/test_gpu_lookahead.py > gpurun_out/r03af/t.log 2>&1 || { echo T_FAIL; tail -30 gpurun_out/r03af/t.log; exit 1; }
tail -1 gpurun_out/r03af/t.log
for v in 1 2; do
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline --no-eager-window --no-pivot-window --steps 100 --warmup 10 > gpurun_out/r03af/c2.json 2> gpurun_out/r03af/c2.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03af/c2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03af/c2.json'));print('c2', round(d['value']), d['ms_per_step'])"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > gpurun_out/r03af/c3.json 2> gpurun_out/r03af/c3.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03af/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03af/c3.json'));print('c3', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
