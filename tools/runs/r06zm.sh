#!/bin/bash
# r06zm: the final build's bench lines and the profiles behind them: the default bench (as the driver runs it),
# its rocprofv3 kernel-trace stats, one PMC pass each for FETCH_SIZE and WRITE_SIZE of the tableau pass, and the
# C5 line
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zm; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('default', round(d['value']), 'frac', round(r['frac'],3), 'pass_ms', round(r['launch_ms'],3), 'cpu', d['cpu_baseline'] and d['cpu_baseline'].get('value'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/trace_bench.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/pmc_write.json 2> $O/pmc_write.err || { tail -20 $O/pmc_write.err; exit 1; }
cd $R
python3 tools/pmc_summary.py $O pass_q_kernel $O/c3_pass_pmc_traffic.json "final round-6 build: condensed C3, form 23 (4-row groups) on 192 CUs" > /dev/null || exit 1
python3 -c "import json; d=json.load(open('$O/c3_pass_pmc_traffic.json')); print('pmc', d['traffic_bytes_per_launch']/1e9, 'GB/launch', 'trace avg ms', d['trace_avg_ns']/1e6)"
timeout -k 10 300 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo FAIL c5; tail -20 $O/bench_c5.err; exit 1; }
tail -1 $O/bench_c5.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', round(d['value']), 'wall', round(d['wall_lps_per_s']))"
echo done
