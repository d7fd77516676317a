#!/bin/bash
# r05ab: unbounded LP through the peer exchange (incl. K = 64 with lookahead)
set -o pipefail
O=gpurun_out/r05ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest "tests/test_gpu_peer.py::test_peer_exchange_unbounded" -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo FAIL; grep -E "Error|assert" $O/tests.log | head -10; tail -5 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" $O/tests.log
