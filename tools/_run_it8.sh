#!/bin/bash
# K = 32 pass: form 4 (2 doubles x 2 rows per lane) across row bands vs the form-3 default.
set -o pipefail
O=gpurun_out/it8
mkdir -p $O
timeout -k 10 500 python tools/tune_defer.py --ks 32 --forms 3,4 --rbs 128,256,512 --nts 1 --occs 0 --rounds 5 > $O/tune_k32_form4_rb.txt 2>&1 && \
echo "it8 done"
