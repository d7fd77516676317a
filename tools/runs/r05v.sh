#!/bin/bash
# r05v: the rank geometries of the N = 2 and N = 4 scaling runs as 2 / 4 processes on one GPU (C3 split, oracle stops
# rank_split_c3), with the rest of the rank-process tests
set -o pipefail
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_gpu_ranks.py -x -v --timeout 600 --timeout-method thread > $O/ranks.log 2>&1 || { echo FAIL ranks; tail -40 $O/ranks.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/ranks.log
