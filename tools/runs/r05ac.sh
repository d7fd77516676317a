#!/bin/bash
# r05ac: C2 (BASELINE configs[1], 4096 x 8192, K = 16, no lookahead by default) with lookahead forced on, now that
# the chain and the pass can run on disjoint CU masks (round 2 measured lookahead losing here without them)
set -o pipefail
O=gpurun_out/r05ac; mkdir -p $O
run() {  # tag args env...
timeout -k 10 300 env "${@:3}" python -u bench.py --workload c2 --no-cpu-baseline --no-eager-window --no-pivot-window $2 > $O/$1.json 2> $O/$1.err || { echo FAIL $1; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); b=d.get('block',{}); g=d['geometry']
print('$1', round(d['value']), 'K', g.get('K'), 'form', g.get('form'), 'la', b.get('lookahead'), 'cus', b.get('chain_cus'), 'pass', b.get('pass_ms'))"
}
for r in a b; do
run def$r "" X=0 && run la$r "--lookahead 1" X=0 && run la_c64$r "--lookahead 1" DLP_CHAIN_CUS=64 && run la_c192$r "--lookahead 1" DLP_CHAIN_CUS=192 \
 && run la_c0$r "--lookahead 1" DLP_CHAIN_CUS=0 && run la_k32$r "--lookahead 1 --defer 32" X=0 && run la_k8$r "--lookahead 1 --defer 8" X=0 || exit 1
done
