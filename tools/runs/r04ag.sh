#!/bin/bash
# r04ag: under the CU split, the form-23 (LDS-ring) pass instead of form 21
set -o pipefail
O=gpurun_out/r04ag; mkdir -p $O
run() {  # workload tag args...
timeout -k 10 300 python -u bench.py --workload $1 --no-cpu-baseline --no-eager-window --no-pivot-window "${@:3}" > $O/$1_$2.json 2> $O/$1.err || { echo FAIL $1 $2; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 $2', round(d['value']), 'form', d['geometry']['form'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'cus', b.get('chain_cus'))"
}
for w in c3r4 c3r2 c3r8; do
run $w f21 && run $w f23 --form 23 && run $w f21b && run $w f23b --form 23 || exit 1
done
