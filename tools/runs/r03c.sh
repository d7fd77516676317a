#!/bin/bash
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03c; mkdir -p $OUT
timeout -k 10 420 python -u -m pytest tests/test_gpu_peer.py -v --timeout 120 --timeout-method thread \
   -k "not c3_row_partition" > $OUT/peer_tests.txt 2>&1; rc=$?
tail -8 $OUT/peer_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/clock_probe.sh r03c_clk || exit 1
grep -h "sclk\|Power\|use" gpurun_out/r03c_clk/clk_smi.txt | sort | uniq -c | sort -rn | head -20
