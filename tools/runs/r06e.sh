#!/bin/bash
# r06e: condensed C3 bench and its kernel trace (per-pivot chain timeline), after moving the pivot-row
# kernels' restart handling into their replay loops; then the lookahead / deferred / large tests
set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window > $O/bench.json 2> $O/bench.err || { echo FAIL bench; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); r=d['roofline']
print('c3', round(d['value']), 'ms/step', round(d['ms_per_step'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'parity', (d.get('pivot_log_vs_oracle') or {}).get('bit_identical'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/prof_bench.json 2> $O/prof_bench.err || { echo FAIL prof; tail -20 $O/prof_bench.err; exit 1; }
K=$(find $O/prof -name "*kernel_trace.csv" | head -1); S=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp $S $O/c3_kernel_stats.csv
python3 tools/kernel_timeline.py $K 3 > $O/timeline.json
rm -f $K
python3 - <<'PY'
import json
t=json.load(open('gpurun_out/r06e/timeline.json'))
for b in t:
    print('block', b['block_us'], 'pass', b['pass_us'], 'pivots', b['pivots'], 'during pass', b['pivots_during_pass'], 'reset', b.get('reset_cols_us'))
    print(' ratio', b['ratio_us'][:6], '...', b['ratio_us'][-6:])
    print(' prow ', b['prow_us'][:6], '...', b['prow_us'][-6:])
    print(' period', b['period_us'][:6], '...', b['period_us'][-6:])
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_lookahead.py tests/test_gpu_defer.py tests/test_gpu_large.py -v --timeout 300 --maxfail 10 --timeout-method thread > $O/tests.log 2>&1; rc=$?
grep -E "FAILED|passed|failed" $O/tests.log | tail -12
exit $rc
