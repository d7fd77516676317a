#!/bin/bash
# r04d: C5 DPP wave-minimum patch (tools/experiments/c5_dpp_wave_min.patch) vs the shipped kernel
set -o pipefail
O=gpurun_out/r04d; mkdir -p $O
for sh in "64 128" "64 64"; do timeout -k 10 120 python -u tools/c5_run.py $sh 5 >> $O/c5_base.json 2>> $O/err.log || { echo BASE_FAIL; tail $O/err.log; exit 1; }; done
cat $O/c5_base.json
cp tools/bin/libdlp_c5dpp.so distributedlpsolver_amd/libdlp.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_large.py -k c5 > $O/dpp_tests.log 2>&1 || { echo DPP_TEST_FAIL; grep -E "FAIL|assert" $O/dpp_tests.log | head; tail -20 $O/dpp_tests.log; exit 1; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k batched >> $O/dpp_tests.log 2>&1 || { echo DPP_TEST_FAIL2; grep -E "FAIL|assert" $O/dpp_tests.log | head; tail -20 $O/dpp_tests.log; exit 1; }
grep -E "passed|failed" $O/dpp_tests.log
for sh in "64 128" "64 64"; do timeout -k 10 120 python -u tools/c5_run.py $sh 5 >> $O/c5_dpp.json 2>> $O/err.log || { echo DPP_FAIL; tail $O/err.log; exit 1; }; done
cat $O/c5_dpp.json
