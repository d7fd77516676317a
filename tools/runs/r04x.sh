#!/bin/bash
# r04x: disjoint CU masks, fine sweep around the best splits, alternating with the unmasked base
set -o pipefail
O=gpurun_out/r04x; mkdir -p $O
run() {  # workload tag env...
timeout -k 10 300 env "${@:3}" python -u bench.py --workload $1 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1_$2.json 2> $O/$1.err || { echo FAIL $1 $2; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 $2', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3))"
}
run c3r8 base X=0 && run c3r8 cus112 DLP_CHAIN_CUS=112 && run c3r8 cus128 DLP_CHAIN_CUS=128 && run c3r8 cus144 DLP_CHAIN_CUS=144 && run c3r8 base2 X=0 && run c3r8 cus128b DLP_CHAIN_CUS=128
run c3r4 base X=0 && run c3r4 cus80 DLP_CHAIN_CUS=80 && run c3r4 cus96 DLP_CHAIN_CUS=96 && run c3r4 cus112 DLP_CHAIN_CUS=112 && run c3r4 base2 X=0 && run c3r4 cus96b DLP_CHAIN_CUS=96
run c3r2 base X=0 && run c3r2 cus48 DLP_CHAIN_CUS=48 && run c3r2 cus64 DLP_CHAIN_CUS=64 && run c3r2 cus80 DLP_CHAIN_CUS=80 && run c3r2 base2 X=0 && run c3r2 cus64b DLP_CHAIN_CUS=64
