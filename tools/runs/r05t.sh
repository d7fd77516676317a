#!/bin/bash
# r05t: the rank geometries (chain on CUs of its own, latency-bound) with the register ratio replay (DLP_MID_CHAIN=1,
# 2 x 16 coefficient loads in flight per lane) and with the chain's LDS rings 16 deep (DLP_CHAIN_RING=16); alternating
set -o pipefail
O=gpurun_out/r05t; mkdir -p $O
run() {  # tag workload env...
timeout -k 10 300 env "${@:3}" python -u bench.py --workload $2 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1.json 2> $O/$1.err || { echo FAIL $1; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'form', d['geometry']['form'])"
}
for r in a b; do
for w in c3r8 c3r4; do
run ${w}_def$r $w X=0 && run ${w}_mid$r $w DLP_MID_CHAIN=1 && run ${w}_r16$r $w DLP_CHAIN_RING=16 || exit 1
done
done
