#!/bin/bash
# r04an: the one-launch peer pivot on the CU split (DLP_PEER_ONELAUNCH A/B)
set -o pipefail
O=gpurun_out/r04an; mkdir -p $O
run() {  # workload tag env...
timeout -k 10 300 env "${@:3}" python -u bench.py --workload $1 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/$1_$2.json 2> $O/$1.err || { echo FAIL $1 $2; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 $2', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'cus', b.get('chain_cus'))"
}
for w in c3r8 c3r4; do
run $w two X=0 && run $w one DLP_PEER_ONELAUNCH=1 && run $w two2 X=0 && run $w one2 DLP_PEER_ONELAUNCH=1 || exit 1
done
