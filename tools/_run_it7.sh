#!/bin/bash
# K = 32 pass at 256-row bands: cache policy (nt) and form 3 vs form 4 (2 doubles x 2 rows per lane).
set -o pipefail
O=gpurun_out/it7
mkdir -p $O
timeout -k 10 500 python tools/tune_defer.py --ks 32 --forms 3,4 --rbs 256 --nts 0,1 --occs 0 --rounds 4 > $O/tune_k32_nt_form.txt 2>&1 && \
echo "it7 done"
