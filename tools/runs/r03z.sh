#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03z
cd /root/repo
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_peer.py > gpurun_out/r03z/peer.log 2>&1 || { echo PEER_FAIL; tail -40 gpurun_out/r03z/peer.log; exit 1; }
grep -E "k64|passed|failed" gpurun_out/r03z/peer.log | tail -6
