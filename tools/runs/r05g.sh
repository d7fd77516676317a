#!/bin/bash
# r05g: C3 with the chain on CUs of its own (DLP_CHAIN_CUS) and the MFMA pass (form 22) on the rest, vs the
# default (form 21, no split) and form 23 on the split; alternating
set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
run() {  # tag args env...
timeout -k 10 300 env "${@:3}" python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window $2 > $O/c3_$1.json 2> $O/c3_$1.err || { echo FAIL $1; tail -20 $O/c3_$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'frac', round(d['roofline']['frac'],4), 'form', d['geometry']['form'], 'cus', b['chain_cus'])"
}
for r in a b; do
run def$r "" X=0 && run f22c32$r "--form 22" DLP_CHAIN_CUS=32 && run f22c64$r "--form 22" DLP_CHAIN_CUS=64 && run f23c32$r "--form 23" DLP_CHAIN_CUS=32 && run f21c32$r "--form 21" DLP_CHAIN_CUS=32 || exit 1
done
bash tools/runs/r05h.sh
