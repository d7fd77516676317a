#!/bin/bash
# r06h: FETCH_SIZE calibration per load type (known-byte read streams), then the condensed C3 default
# bench (driver protocol, CPU baselines), its kernel trace and the PMC passes of its tableau pass
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06h; mkdir -p $O
mkdir -p /tmp/fc && hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/fc/fetch_calib tools/fetch_calib.hip || exit 1
cd /tmp && export TMPDIR=/tmp
for k in b64 b128 glds; do
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/calib_$k -o run -- /tmp/fc/fetch_calib $k 4 > $O/calib_$k.txt 2> $O/calib_$k.err || { echo FAIL calib $k; tail -5 $O/calib_$k.err; exit 1; }
  tail -1 $O/calib_$k.txt
done
cd $R
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo FAIL bench; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']; c=d['cpu_baseline']
print('c3', round(d['value']), 'ms/step', round(d['ms_per_step'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'parity', d['pivot_log_vs_oracle']['bit_identical'], 'cpu', round(c['value'],2), round(c['like_for_like']['value'],1), 'eager', round(d['rank1_update_roofline']['frac'],3))"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window > $O/trace_bench.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/pmc_write.json 2> $O/pmc_write.err || { tail -20 $O/pmc_write.err; exit 1; }
cd $R
timeout -k 10 300 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo FAIL c5; tail -20 $O/bench_c5.err; exit 1; }
echo done
