#!/bin/bash
# r06d: condensed tableau vs full on the bench: C3 default line (condensed), C3 with DLP_CONDENSED=0, C2 both,
# then a rocprofv3 kernel trace of the condensed C3 bench
set -o pipefail
O=gpurun_out/r06d; mkdir -p $O
run() {  # tag env... -- args
  tag=$1; shift
  timeout -k 10 400 env "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$tag', round(d['value']), 'ms/step', round(d['ms_per_step'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'form', d['geometry']['form'], 'ld', d['geometry']['ld'], 'parity', (d.get('pivot_log_vs_oracle') or {}).get('bit_identical'))"
}
run c3_cond X=1 python -u bench.py --no-cpu-baseline --no-eager-window || exit 1
run c3_full DLP_CONDENSED=0 python -u bench.py --no-cpu-baseline --no-eager-window || exit 1
run c2_cond X=1 python -u bench.py --workload c2 --steps 100 --warmup 10 --no-cpu-baseline --no-eager-window || exit 1
run c2_full DLP_CONDENSED=0 python -u bench.py --workload c2 --steps 100 --warmup 10 --no-cpu-baseline --no-eager-window || exit 1
run c3_cond2 X=1 python -u bench.py --no-cpu-baseline --no-eager-window || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o c3 -- python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/prof_bench.json 2> $O/prof_bench.err || { echo FAIL prof; tail -20 $O/prof_bench.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
