#!/bin/bash
# r06b: condensed tableau, first GPU check: deferred / lookahead / parity tests
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_lookahead.py tests/test_gpu_parity.py -v --timeout 120 --maxfail 30 --timeout-method thread > $O/t1.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t1.log | tail -30
if [ $rc -ne 0 ]; then grep -E "^E " $O/t1.log | head -30; exit 1; fi
