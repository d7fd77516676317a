#!/bin/bash
# r06zt: final round-6 build: the whole GPU suite, then smoke()
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zt; mkdir -p $O
timeout -k 10 1050 python -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread --durations=25 > $O/suite.log 2>&1
rc=$?; tail -4 $O/suite.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/suite.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
echo done
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('default', round(d['value']), 'frac', round(r['frac'],3), 'pass_ms', round(r['launch_ms'],3), 'parity', d['pivot_log_vs_oracle']['bit_identical'])"
