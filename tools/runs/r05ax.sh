#!/bin/bash
# r05ax: c3r2 (pass-bound at 16,384 rows per rank) with the form-23 pass's ring depth 6 / 8 and its workgroups held to
# 2 per CU (DLP_PASS_LDS), alternating on one box
set -o pipefail
O=gpurun_out/r05ax; mkdir -p $O
run() {  # tag env...
timeout -k 10 300 env "${@:2}" python -u bench.py --workload c3r2 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1.json 2> $O/$1.err || { echo FAIL $1; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'form', d['geometry']['form'], 'cus', b.get('chain_cus'))"
}
for r in a b; do
run def$r X=0 && run q6$r DLP_Q_DEPTH=6 && run q8$r DLP_Q_DEPTH=8 && run l56$r DLP_PASS_LDS=57344 && run q3$r DLP_Q_DEPTH=3 || exit 1
done
