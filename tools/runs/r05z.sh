#!/bin/bash
# r05z: chain CU count at the rank geometries again, now with 128-lane ratio workgroups (fewer CUs may suffice for the
# chain); alternating
set -o pipefail
O=gpurun_out/r05z; mkdir -p $O
run() {  # tag workload env...
timeout -k 10 300 env "${@:3}" python -u bench.py --workload $2 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1.json 2> $O/$1.err || { echo FAIL $1; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'form', d['geometry']['form'], 'cus', b.get('chain_cus'))"
}
for r in a b; do
for w in c3r8 c3r4; do
run ${w}_def$r $w X=0 && run ${w}_c64$r $w DLP_CHAIN_CUS=64 && run ${w}_c96$r $w DLP_CHAIN_CUS=96 && run ${w}_c160$r $w DLP_CHAIN_CUS=160 || exit 1
done
done
