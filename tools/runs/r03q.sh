#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03ad
cd /root/repo
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03ad/gpu_suite.log 2>&1 || { echo SUITE_FAIL; tail -40 gpurun_out/r03ad/gpu_suite.log; exit 1; }
tail -3 gpurun_out/r03ad/gpu_suite.log
