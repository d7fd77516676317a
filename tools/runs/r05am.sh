#!/bin/bash
# r05am: final round-5 checkpoint on the shipped build: full GPU suite, smoke, default bench (driver protocol), the c5
# line, a rocprofv3 kernel trace of the default bench, then the PMC FETCH_SIZE / WRITE_SIZE passes of the C3 pass
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05am; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/suite.log 2>&1 || { echo FAIL suite; tail -40 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { echo FAIL smoke; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo FAIL bench; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo FAIL c5; tail -20 $O/bench_c5.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('c3', round(d['value']), 'pass', d['roofline']['launch_ms'], d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('like_for_like',{}).get('value'))
d=json.loads(open('$O/bench_c5.json').read().strip().splitlines()[-1]); print('c5', round(d['value']), d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window > $O/trace_bench.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/pmc_write.json 2> $O/pmc_write.err || { tail -20 $O/pmc_write.err; exit 1; }
echo done
