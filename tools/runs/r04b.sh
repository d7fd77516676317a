#!/bin/bash
# r04b: exchange auto / fallback, late rank, C3 8-rank split with lookahead (tests)
set -o pipefail
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_peer.py tests/test_gpu_faults.py > $O/peer.log 2>&1 || { echo PEER_FAIL; grep -E "FAIL|Error|assert" $O/peer.log | head -30; tail -30 $O/peer.log; exit 1; }
tail -3 $O/peer.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_lookahead.py tests/test_gpu_parity.py tests/test_gpu_general.py > $O/rest.log 2>&1 || { echo REST_FAIL; grep -E "FAIL|Error|assert" $O/rest.log | head -30; tail -30 $O/rest.log; exit 1; }
tail -3 $O/rest.log
