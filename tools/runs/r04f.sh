#!/bin/bash
# r04f: DPP block reductions everywhere: full GPU suite, c3r8 + C3 benches, chain stamps
set -o pipefail
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" $O/suite.log | head -30; tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 240 python -u bench.py --workload c3r8 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/c3r8_auto.json 2> $O/c3r8.err || { echo C3R8_FAIL; tail -20 $O/c3r8.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3r8_auto.json').read().strip().splitlines()[-1]); b=d['block']
print('c3r8 auto', round(d['value']), d['exchange'], 'la', b['lookahead'], 'form', d['geometry']['form'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'chain', b['chain_us_per_pivot'])"
DLP_LEAN_LCH=0 timeout -k 10 200 python -u tools/chain_stamps.py --workload c3r8 --exchange peer --lookahead 1 > $O/stamps_c3r8.json 2>&1 || { echo STAMP_FAIL; tail -20 $O/stamps_c3r8.json; exit 1; }
DLP_LEAN_LCH=0 timeout -k 10 200 python -u tools/chain_stamps.py > $O/stamps_c3.json 2>&1 || { echo STAMP_FAIL; tail -20 $O/stamps_c3.json; exit 1; }
python3 -c "
import json
for f in ('stamps_c3r8','stamps_c3'):
    d=json.load(open('$O/'+f+'.json')); print(f, round(d['bench_value']), {k: round(v,2) for k,v in d['median_us'].items()})"
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window > $O/c3_$i.json 2> $O/c3.err || { echo C3_FAIL; tail -20 $O/c3.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_$i.json').read().strip().splitlines()[-1])
print('c3', round(d['value']), d['ms_per_step'], d['roofline']['launch_ms'], d['roofline']['frac'], d['pivot_log_vs_oracle']['bit_identical'])"
done
DLP_TRACE_CREATE=1 timeout -k 10 120 python -u tools/c1_overhead.py > $O/c1_overhead.json 2> $O/c1_stages.txt || { echo C1_FAIL; tail $O/c1_stages.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/c1prof -o run -- python3 $GRAFT_REPO_ROOT/tools/c1_overhead.py > $GRAFT_REPO_ROOT/$O/c1_prof.json 2>&1 || { echo C1PROF_FAIL; exit 1; }
cd $GRAFT_REPO_ROOT
python3 -c "
import csv,glob
f=glob.glob('$O/c1prof/**/*kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]: print(r['Name'].replace('void dlp::(anonymous namespace)::','').split('(')[0][:50], r['Calls'], round(float(r['AverageNs'])/1e3,2))"
echo r04f done
