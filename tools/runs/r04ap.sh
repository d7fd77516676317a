#!/bin/bash
# r04ap: the full GPU suite + smoke + bench_extra (C1 / C4 / C5 / f1) after the C5 change
set -o pipefail
O=gpurun_out/r04ap; mkdir -p $O
timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_suite.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" $O/gpu_suite.log | head -30; tail -30 $O/gpu_suite.log; exit 1; }
tail -1 $O/gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u tools/bench_extra.py > $O/extra.json 2> $O/extra.err || { echo EXTRA_FAIL; tail $O/extra.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/extra.json'))
for k,v in d.items(): print(k, {a: b for a, b in v.items() if isinstance(b, (int, float))} if isinstance(v, dict) else v)" | cut -c1-300
