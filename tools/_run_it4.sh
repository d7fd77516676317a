#!/bin/bash
# Form 6 (form 3 at >= 5 waves/SIMD): parity, then an interleaved A/B against form 3 at K = 32.
set -o pipefail
O=gpurun_out/it4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_defer.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 && \
timeout -k 10 400 python tools/tune_defer.py --ks 32 --forms 3,6 --rbs 128,256 --occs 0 --rounds 4 > $O/tune_k32_forms36.txt 2>&1 && \
timeout -k 10 400 python tools/tune_defer.py --ks 48,64 --forms 3,6 --rbs 256 --occs 0 --rounds 2 > $O/tune_k4864_forms36.txt 2>&1 && \
echo "it4 done"
