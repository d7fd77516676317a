#!/bin/bash
# K = 32 pass: wider row bands (fewer re-reads of the P block per column tile).
set -o pipefail
O=gpurun_out/it6
mkdir -p $O
timeout -k 10 400 python tools/tune_defer.py --ks 32 --forms 3 --rbs 256,512,1024 --occs 0 --rounds 4 > $O/tune_k32_rb.txt 2>&1 && \
echo "it6 done"
