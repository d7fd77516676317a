#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03ag
cd /root/repo
for nt in 1 1; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --nontemporal $nt > gpurun_out/r03ag/b.json 2> gpurun_out/r03ag/b.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03ag/b.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03ag/b.json'));print('nt=$nt', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
done
