#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03final
cd /root/repo
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03final/gpu_suite.log 2>&1 || { echo SUITE_FAIL; tail -40 gpurun_out/r03final/gpu_suite.log; exit 1; }
tail -2 gpurun_out/r03final/gpu_suite.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03final/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/r03final/smoke.log; exit 1; }
tail -1 gpurun_out/r03final/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/r03final/bench_default.json 2> gpurun_out/r03final/bench_default.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03final/bench_default.err; exit 1; }
cat gpurun_out/r03final/bench_default.json
