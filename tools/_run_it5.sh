#!/bin/bash
# After the P-row bound fix (non-power-of-two K): deferred parity, then K = 48 / 64 / 32 at C3.
set -o pipefail
O=gpurun_out/it5
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_defer.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 && \
timeout -k 10 400 python tools/tune_defer.py --ks 32,48 --forms 3 --rbs 256 --occs 0 --rounds 3 > $O/tune_k32_k48.txt 2>&1 && \
echo "it5 done"
