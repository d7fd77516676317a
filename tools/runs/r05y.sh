#!/bin/bash
# r05y: C3's 8-rank split as 8 rank processes on one GPU (each chain on its own 32 CUs), against the oracle's stops
set -o pipefail
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 900 python -u -m pytest "tests/test_gpu_ranks.py::test_c3_rank_processes" -x -v --timeout 600 --timeout-method thread > $O/ranks.log 2>&1 || { echo FAIL ranks; grep -E "Error|error" $O/ranks.log | head -5; tail -5 $O/ranks.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/ranks.log
