#!/bin/bash
# r05m: C3 default (form 21, no split) vs the chain on 32 CUs of its own (auto form 23 on the other 224),
# alternating 3 x, on whatever box this call lands on (round 4 and round 5 disagreed by box)
set -o pipefail
O=gpurun_out/r05m_$(date +%H%M%S); mkdir -p $O
run() {  # tag env...
timeout -k 10 300 env "${@:2}" python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/c3_$1.json 2> $O/c3_$1.err || { echo FAIL $1; tail -20 $O/c3_$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'form', d['geometry']['form'], 'cus', b['chain_cus'])"
}
for r in a b c; do
run def$r X=0 && run c32$r DLP_CHAIN_CUS=32 || exit 1
done
