#!/bin/bash
# r05q: the full GPU suite after the 128-lane ratio policy, then smoke and the default bench
set -o pipefail
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || { echo FAIL suite; tail -40 $O/suite.log; exit 1; }
tail -3 $O/suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { echo FAIL smoke; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo FAIL bench; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('c3', round(d['value']), 'pass', d['roofline']['launch_ms'], d['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('like_for_like',{}).get('value'))"
