#!/bin/bash
# r04l: block size K at the rank geometries (lookahead forced on for K < 64)
set -o pipefail
O=gpurun_out/r04l; mkdir -p $O
run() {  # workload defer lookahead tag
timeout -k 10 300 python -u bench.py --workload $1 --defer $2 --lookahead $3 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1_k$2_la$3.json 2> $O/$1.err || { echo FAIL $1 $2 $3; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_k$2_la$3.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 K', d['K'], 'la', b['lookahead'], 'form', d['geometry']['form'], round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'chain', b['chain_us_per_pivot'])"
}
run c3r8 32 1 && run c3r8 32 0 && run c3r8 64 1 && run c3r8 16 1 && run c3r4 32 1 && run c3r4 64 1 && run c3r2 32 1 && run c3r2 64 1
