#!/bin/bash
# r05k: the cross-process stall test at the shipped rank geometry + the rank-path tests on the current build
set -o pipefail
O=gpurun_out/r05k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ranks.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo FAIL tests; tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/tests.log | tail -10
