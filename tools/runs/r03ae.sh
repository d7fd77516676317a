#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03ae
cd /root/repo
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_defer.py > gpurun_out/r03ae/defer.log 2>&1 || { echo DEFER_FAIL; tail -30 gpurun_out/r03ae/defer.log; exit 1; }
tail -1 gpurun_out/r03ae/defer.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03ae/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r03ae/smoke.log; exit 1; }
tail -2 gpurun_out/r03ae/smoke.log
