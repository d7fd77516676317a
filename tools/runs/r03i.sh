#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03i
cd /root/repo
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lookahead.py tests/test_isa.py > gpurun_out/r03i/la.log 2>&1 || { echo LA_FAIL; tail -30 gpurun_out/r03i/la.log; exit 1; }
tail -3 gpurun_out/r03i/la.log
timeout -k 10 180 python -u tools/chain_stamps.py > gpurun_out/r03i/stamps.json 2>&1 || { echo STAMP_FAIL; tail -20 gpurun_out/r03i/stamps.json; exit 1; }
cat gpurun_out/r03i/stamps.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03i/bench.json 2> gpurun_out/r03i/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r03i/bench.err; exit 1; }
cat gpurun_out/r03i/bench.json
