#!/bin/bash
# r05ad: C5 phase stamps (LP 0, first 64 pivots) of the register-resident batched kernel, full batch and one LP per CU
set -o pipefail
O=gpurun_out/r05ad; mkdir -p $O
for a in "64 128 4096" "64 128 256" "64 64 4096" "64 64 256"; do
t=$(echo $a | tr ' ' _)
timeout -k 10 120 python -u tools/batch_stamps.py $a > $O/stamps_$t.json 2> $O/stamps_$t.err || { echo FAIL $t; tail -5 $O/stamps_$t.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/stamps_$t.json')); print('$t', round(d['kernel_ms'],3), {k: round(v,2) for k,v in d['median_us'].items()})"
done
