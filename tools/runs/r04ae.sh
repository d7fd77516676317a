#!/bin/bash
# r04ae: C2 (4k x 8k, K = 16) with lookahead and the disjoint CU split
set -o pipefail
O=gpurun_out/r04ae; mkdir -p $O
run() {  # tag args/env...
timeout -k 10 300 env ${ENVV} python -u bench.py --workload c2 --steps 100 --warmup 10 --no-cpu-baseline --no-eager-window --no-pivot-window "${@:2}" > $O/c2_$1.json 2> $O/c2.err || { echo FAIL $1; tail -20 $O/c2.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c2_$1.json').read().strip().splitlines()[-1]); b=d['block']
print('c2 $1', round(d['value']), 'K', d['K'], 'la', b['lookahead'], 'block', round(b['ms'],4), 'pass', round(b['pass_ms'],4), 'cus', b.get('chain_cus'), 'bit', (d.get('pivot_log_vs_oracle') or {}).get('bit_identical'))"
}
ENVV="X=0" run base && ENVV="X=0" run la1 --lookahead 1 && ENVV="DLP_CHAIN_CUS=64" run la1_c64 --lookahead 1 && ENVV="DLP_CHAIN_CUS=96" run la1_c96 --lookahead 1 && ENVV="DLP_CHAIN_CUS=160" run la1_c160 --lookahead 1 && ENVV="DLP_CHAIN_CUS=192" run la1_c192 --lookahead 1 && ENVV="X=0" run k32la1 --lookahead 1 --defer 32 && ENVV="DLP_CHAIN_CUS=64" run k32la1_c64 --lookahead 1 --defer 32 && ENVV="DLP_CHAIN_CUS=160" run k32la1_c160 --lookahead 1 --defer 32 && ENVV="X=0" run base2
