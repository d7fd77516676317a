#!/bin/bash
# r04aq: K = 32 with lookahead on the CU split at the rank geometries
set -o pipefail
O=gpurun_out/r04aq; mkdir -p $O
run() {  # workload tag args...
timeout -k 10 300 python -u bench.py --workload $1 --no-cpu-baseline --no-eager-window --no-pivot-window "${@:3}" > $O/$1_$2.json 2> $O/$1.err || { echo FAIL $1 $2; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 $2', round(d['value']), 'K', d['K'], 'form', d['geometry']['form'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'cus', b.get('chain_cus'))"
}
for w in c3r8 c3r4; do
run $w k64 && run $w k32 --defer 32 --lookahead 1 || exit 1
done
DLP_CHAIN_CUS=160 run c3r8 k32c160 --defer 32 --lookahead 1 && DLP_CHAIN_CUS=96 run c3r8 k32c96 --defer 32 --lookahead 1
