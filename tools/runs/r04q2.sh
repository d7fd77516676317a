#!/bin/bash
# r04q (second half): the GPU suite from test_gpu_large on, C1 end to end
set -o pipefail
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_large.py tests/test_gpu_lookahead.py tests/test_gpu_parity.py tests/test_gpu_peer.py tests/test_gpu_rowblock.py tests/test_mw.py -m gpu > $O/suite2.log 2>&1 || { echo SUITE_FAIL; grep -E "FAIL|Error|assert" $O/suite2.log | head -30; tail -30 $O/suite2.log; exit 1; }
tail -1 $O/suite2.log
DLP_TRACE_CREATE=1 timeout -k 10 120 python -u tools/c1_probe.py > $O/c1_probe.txt 2>&1 || { echo C1_FAIL; tail $O/c1_probe.txt; exit 1; }
grep -v "^dlp stage" $O/c1_probe.txt
timeout -k 10 120 python -u tools/c1_overhead.py > $O/c1_overhead.json 2> $O/c1.err || { echo C1O_FAIL; tail $O/c1.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/c1_overhead.json'))
for k,v in d.items(): print('c1', k, v['pivots'], [round(x,2) for x in v['solve_ms']], {a: round(b,3) for a,b in v['parts'][-1].items()})"
timeout -k 10 200 python -u tools/bench_extra.py > $O/extra.json 2> $O/extra.err || { echo EXTRA_FAIL; tail $O/extra.err; exit 1; }
tail -c 1500 $O/extra.json
