#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03ac
cd /root/repo
for v in 1 2; do
timeout -k 10 300 python -u bench.py --workload c2 --no-cpu-baseline --no-eager-window --no-pivot-window --steps 100 --warmup 10 > gpurun_out/r03ac/c2.json 2> gpurun_out/r03ac/c2.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03ac/c2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03ac/c2.json'));print('c2', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['geometry'], d['pivot_log_vs_oracle'])"
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /root/repo/gpurun_out/r03ac/trace -o run -- python3 /root/repo/bench.py --workload c2 --no-cpu-baseline --no-eager-window --no-pivot-window --steps 100 --warmup 10 > /root/repo/gpurun_out/r03ac/trace.json 2> /root/repo/gpurun_out/r03ac/trace.err || { echo TRACE_FAIL; tail -5 /root/repo/gpurun_out/r03ac/trace.err; exit 1; }
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('/root/repo/gpurun_out/r03ac/trace/run_kernel_stats.csv')))
for r in rows[:8]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us', r['Percentage'])
PY
