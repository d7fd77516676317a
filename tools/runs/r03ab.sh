#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03ab
cd /root/repo
timeout -k 10 120 python -u tools/batch_stamps.py 64 128 > gpurun_out/r03ab/st128.json 2>&1 || { echo ST_FAIL; tail -20 gpurun_out/r03ab/st128.json; exit 1; }
cat gpurun_out/r03ab/st128.json
timeout -k 10 120 python -u tools/batch_stamps.py 64 64 > gpurun_out/r03ab/st64.json 2>&1 || { echo ST_FAIL; tail -20 gpurun_out/r03ab/st64.json; exit 1; }
cat gpurun_out/r03ab/st64.json
