#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03aa
cd /root/repo
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "batched" > gpurun_out/r03aa/bt.log 2>&1 || { echo BT_FAIL; tail -40 gpurun_out/r03aa/bt.log; exit 1; }
tail -2 gpurun_out/r03aa/bt.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_large.py -k "c5" > gpurun_out/r03aa/c5.log 2>&1 || { echo C5_FAIL; tail -40 gpurun_out/r03aa/c5.log; exit 1; }
tail -2 gpurun_out/r03aa/c5.log
for v in 0 1; do for mn in "64 128" "64 64"; do
DLP_BATCH_LDS=$v timeout -k 10 120 python -u tools/c5_run.py $mn 3 > gpurun_out/r03aa/c5_$v.json 2>&1 || { echo RUN_FAIL; tail -20 gpurun_out/r03aa/c5_$v.json; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03aa/c5_$v.json'));print('lds=$v', '$mn', round(d['lps_per_s_kernel']), [r['kernel_ms'] for r in d['runs']], d['runs'][0]['all_optimal'])"
done; done
timeout -k 10 120 python -u tools/batch_stamps.py 64 128 > gpurun_out/r03aa/st128.json 2>&1 || { echo ST_FAIL; tail -20 gpurun_out/r03aa/st128.json; exit 1; }
cat gpurun_out/r03aa/st128.json
