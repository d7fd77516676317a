#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03t
cd /root/repo
for rb in 768 1024 512 768 1024 512; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --rows-per-block $rb > gpurun_out/r03t/bench$rb.json 2> gpurun_out/r03t/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03t/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03t/bench$rb.json'));print('rb=$rb', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'], d['geometry']['rows_per_block'])"
done
