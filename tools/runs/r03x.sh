#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03x
cd /root/repo
for cfg in "21 -1" "23 -1" "23 2" "21 -1" "23 -1" "23 2"; do set -- $cfg
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --form $1 --occupancy $2 > gpurun_out/r03x/b.json 2> gpurun_out/r03x/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03x/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03x/b.json'));print('form $1 occ $2', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['pivot_log_vs_oracle']['bit_identical'])"
done
timeout -k 10 180 python -u tools/chain_stamps.py --form 23 --occupancy 2 > gpurun_out/r03x/stamps23o2.json 2>&1 || { echo STAMP_FAIL; tail -20 gpurun_out/r03x/stamps23o2.json; exit 1; }
cat gpurun_out/r03x/stamps23o2.json
