#!/bin/bash
# r05x: C3 over 4 rank processes on one GPU with disjoint 32-CU chain slices per process (DLP_TEST_CHAIN_CU_FIRST), then
# the rank-process tests
set -o pipefail
O=gpurun_out/r05x; mkdir -p $O
for r in 0; do :; done
timeout -k 10 1000 python -u -m pytest tests/test_gpu_ranks.py -x -v --timeout 600 --timeout-method thread > $O/ranks.log 2>&1 || { echo FAIL ranks; grep -E "Error|error" $O/ranks.log | head -5; tail -5 $O/ranks.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/ranks.log
