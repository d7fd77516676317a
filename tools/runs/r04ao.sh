#!/bin/bash
# r04ao: C5 register kernel without the RHS slot (ceil(n/64) waves per LP): parity, then timings
set -o pipefail
O=gpurun_out/r04ao; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_knobs.py -m gpu -k "batch or c5" > $O/tests.log 2>&1 || { echo TEST_FAIL; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
timeout -k 10 120 python -u tools/c5_run.py 64 128 5 > $O/c5_128_$r.txt 2>&1 || { echo C5FAIL; tail $O/c5_128_$r.txt; exit 1; }
tail -2 $O/c5_128_$r.txt
timeout -k 10 120 python -u tools/c5_run.py 64 64 5 > $O/c5_64_$r.txt 2>&1 || { echo C5FAIL; tail $O/c5_64_$r.txt; exit 1; }
tail -2 $O/c5_64_$r.txt
done
