#!/bin/bash
# r05o: C2 (BASELINE configs[1], K = 16, no lookahead: 17 ratio workgroups of 256 lanes) with 128 / 64-lane ratio
# workgroups; alternating
set -o pipefail
O=gpurun_out/r05o; mkdir -p $O
run() {  # tag env...
timeout -k 10 300 env "${@:2}" python -u bench.py --workload c2 --steps 100 --warmup 10 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/c2_$1.json 2> $O/c2_$1.err || { echo FAIL $1; tail -20 $O/c2_$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c2_$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],4), 'pass', round(b['pass_ms'],4), 'K', d['K'], 'form', d['geometry']['form'], 'chain us', b['chain_us_per_pivot'])"
}
for r in a b; do
run r256$r DLP_RATIO_THREADS=256 && run r128$r DLP_RATIO_THREADS=128 && run r64$r DLP_RATIO_THREADS=64 || exit 1
done
