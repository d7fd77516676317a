#!/bin/bash
# r05aw (second call): c3r2 with 32 and 48 chain CUs (the first call: 128-lane ratio workgroups and 96 chain CUs,
# profiles/r05aw/README.md), alternating on one box
set -o pipefail
O=gpurun_out/r05aw2; mkdir -p $O
run() {  # tag env...
timeout -k 10 300 env "${@:2}" python -u bench.py --workload c3r2 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1.json 2> $O/$1.err || { echo FAIL $1; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'form', d['geometry']['form'], 'cus', b.get('chain_cus'))"
}
for r in a b; do
run def$r X=0 && run c32$r DLP_CHAIN_CUS=32 && run c48$r DLP_CHAIN_CUS=48 || exit 1
done
