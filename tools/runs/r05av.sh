#!/bin/bash
# r05av: final round-5 build (C5 r05at): full GPU suite, smoke, default bench, the c5 line
set -o pipefail
O=gpurun_out/r05av; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/suite.log 2>&1 || { echo FAIL suite; tail -40 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { echo FAIL smoke; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo FAIL bench; tail -20 $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo FAIL c5; tail -20 $O/bench_c5.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('c3', round(d['value']), 'pass', d['roofline']['launch_ms'], d['roofline']['frac'], d['roofline']['traffic_source'])
d=json.loads(open('$O/bench_c5.json').read().strip().splitlines()[-1]); print('c5', round(d['value']), d['roofline']['frac'])"
