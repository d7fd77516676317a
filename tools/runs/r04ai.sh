#!/bin/bash
# r04ai: C3 (P = 1) A/B on one box: form 21 unmasked (default) vs form 23 with the chain on 32 CUs
set -o pipefail
O=gpurun_out/r04ai; mkdir -p $O
run() {  # tag n form
timeout -k 10 300 env DLP_CHAIN_CUS=$2 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --form $3 > $O/c3_$1.json 2> $O/c3.err || { echo FAIL $1; tail -20 $O/c3.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_$1.json').read().strip().splitlines()[-1]); b=d['block']
print('c3 $1', round(d['value']), 'form', d['geometry']['form'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'cus', b.get('chain_cus'), 'bit', d['pivot_log_vs_oracle']['bit_identical'])"
}
for r in 1 2; do
run f21_c0_$r 0 21 && run f23_c32_$r 32 23 && run f21_c32_$r 32 21 && run f23_c64_$r 64 23 || exit 1
done
