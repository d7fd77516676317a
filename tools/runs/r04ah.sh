#!/bin/bash
# r04ah: form 23 under the CU split, chain CUs re-swept
set -o pipefail
O=gpurun_out/r04ah; mkdir -p $O
run() {  # workload tag n args...
timeout -k 10 300 env DLP_CHAIN_CUS=$3 python -u bench.py --workload $1 --no-cpu-baseline --no-eager-window --no-pivot-window --form 23 "${@:4}" > $O/$1_$2.json 2> $O/$1.err || { echo FAIL $1 $2; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 $2', round(d['value']), 'form', d['geometry']['form'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'cus', b.get('chain_cus'))"
}
run c3r8 c128 128 && run c3r8 c144 144 && run c3r8 c160 160 && run c3r8 c176 176 && run c3r8 c192 192 || exit 1
run c3r4 c96 96 && run c3r4 c112 112 && run c3r4 c128 128 && run c3r4 c144 144 && run c3r4 c160 160 || exit 1
run c3r2 c48 48 && run c3r2 c64 64 && run c3r2 c80 80 && run c3r2 c96 96 && run c3r2 c112 112 || exit 1
run c3 c0 0 && run c3 c16 16 && run c3 c32 32 && run c3 c48 48 || exit 1
