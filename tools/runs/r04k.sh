#!/bin/bash
# r04k: C3 (P = 1) row stride sweep for the form-21 lookahead pass (ld = roundup(width, ld_align))
set -o pipefail
O=gpurun_out/r04k; mkdir -p $O
for ld in 65664 65600 65632 65696 65728 65792 65920 65664 66176 65568; do
timeout -k 10 300 python -u bench.py --ld-align $ld --no-cpu-baseline --no-eager-window --no-pivot-window > $O/c3_ld$ld.json 2> $O/c3.err || { echo C3_FAIL $ld; tail -20 $O/c3.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_ld$ld.json').read().strip().splitlines()[-1])
print('ld', d['geometry']['ld'], round(d['value']), round(d['ms_per_step'],3), 'pass', round(d['roofline']['launch_ms'],3), round(d['roofline']['frac'],4), d['pivot_log_vs_oracle']['bit_identical'])"
done
