#!/bin/bash
# r04w: disjoint CU masks, wider splits (DLP_CHAIN_CUS=n)
set -o pipefail
O=gpurun_out/r04w; mkdir -p $O
run() {  # workload tag env...
timeout -k 10 300 env "${@:3}" python -u bench.py --workload $1 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1_$2.json 2> $O/$1.err || { echo FAIL $1 $2; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 $2', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3))"
}
run c3r8 base X=0 && run c3r8 cus128 DLP_CHAIN_CUS=128 && run c3r8 cus160 DLP_CHAIN_CUS=160 && run c3r8 cus192 DLP_CHAIN_CUS=192 && run c3r8 cus224 DLP_CHAIN_CUS=224 && run c3r8 cus128b DLP_CHAIN_CUS=128
run c3r4 base X=0 && run c3r4 cus96 DLP_CHAIN_CUS=96 && run c3r4 cus128 DLP_CHAIN_CUS=128 && run c3r4 cus160 DLP_CHAIN_CUS=160
run c3r2 base X=0 && run c3r2 cus64 DLP_CHAIN_CUS=64 && run c3r2 cus96 DLP_CHAIN_CUS=96 && run c3r2 cus128 DLP_CHAIN_CUS=128
