#!/bin/bash
# r04v: lookahead with the chain and the pass on DISJOINT CU masks (DLP_CHAIN_CUS=n: chain on the top
# n mask bits, pass on the rest)
set -o pipefail
O=gpurun_out/r04v; mkdir -p $O
run() {  # workload tag env...
timeout -k 10 300 env "${@:3}" python -u bench.py --workload $1 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1_$2.json 2> $O/$1.err || { echo FAIL $1 $2; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 $2', round(d['value']), 'la', b['lookahead'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'bit', (d.get('pivot_log_vs_oracle') or {}).get('bit_identical'))"
}
run c3r8 base X=0 && run c3r8 cus16 DLP_CHAIN_CUS=16 && run c3r8 cus32 DLP_CHAIN_CUS=32 && run c3r8 cus64 DLP_CHAIN_CUS=64 && run c3r8 cus96 DLP_CHAIN_CUS=96 && run c3r8 cus128 DLP_CHAIN_CUS=128
run c3r4 base X=0 && run c3r4 cus32 DLP_CHAIN_CUS=32 && run c3r4 cus64 DLP_CHAIN_CUS=64
run c3r2 base X=0 && run c3r2 cus32 DLP_CHAIN_CUS=32

