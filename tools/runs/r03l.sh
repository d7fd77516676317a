#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03l
cd /root/repo
timeout -k 10 180 python -u tools/chain_stamps.py --form 23 > gpurun_out/r03l/stamps23.json 2>&1 || { echo STAMP_FAIL; tail -20 gpurun_out/r03l/stamps23.json; exit 1; }
cat gpurun_out/r03l/stamps23.json
for f in 21 23 21 23; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --form $f > gpurun_out/r03l/bench$f.json 2> gpurun_out/r03l/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03l/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03l/bench$f.json'));print('form=$f', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'], d['config']['lookahead'])"
done
