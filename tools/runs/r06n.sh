#!/bin/bash
# r06n: condensed C3: form-23 pass with 4 rows per group (DLP_Q_U=4, D = 2 / 3) vs the default 2 rows, alternating
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06n; mkdir -p $O
run() {  # tag env...
  tag=$1; shift
  timeout -k 10 300 env "$@" python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'parity', d['pivot_log_vs_oracle']['bit_identical'])"
}
for r in a b; do
run u2_$r X=0 || exit 1
run u4d2_$r DLP_Q_U=4 DLP_Q_DEPTH=2 || exit 1
run u4d3_$r DLP_Q_U=4 DLP_Q_DEPTH=3 || exit 1
done
