#!/bin/bash
# r04am: round-4 final checkpoint: full GPU suite, smoke, default bench (driver protocol, CPU baseline), its
# rocprofv3 kernel stats, the rank-geometry workloads
set -o pipefail
O=gpurun_out/r04am; mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" $O/gpu_suite.log | head -30; tail -30 $O/gpu_suite.log; exit 1; }
tail -1 $O/gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo BENCH_FAIL; tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-400
for w in c3r8 c3r4 c3r2; do
timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-eager-window > $O/$w.json 2> $O/$w.err || { echo FAIL $w; tail -20 $O/$w.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$w.json').read().strip().splitlines()[-1]); b=d['block']
print('$w', round(d['value']), d['exchange'], 'la', b['lookahead'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/bench_prof.json 2> $GRAFT_REPO_ROOT/$O/bench_prof.err || { echo PROF_FAIL; tail -20 $GRAFT_REPO_ROOT/$O/bench_prof.err; exit 1; }
cd $GRAFT_REPO_ROOT
f=$(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1); cp $f $O/kernel_stats.csv
python3 -c "
import csv
for r in list(csv.DictReader(open('$O/kernel_stats.csv')))[:8]: print(r['Name'].replace('void dlp::(anonymous namespace)::','').split('(')[0][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
rm -rf $O/prof
