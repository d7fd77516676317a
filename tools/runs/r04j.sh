#!/bin/bash
# r04j: one-launch peer pivot with s_sleep(8) pollers, A/B against two launches
set -o pipefail
O=gpurun_out/r04j; mkdir -p $O
for w in c3r8 c3r4 c3r8 c3r4; do for one in 1 0; do
DLP_PEER_ONELAUNCH=$one timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-eager-window --no-pivot-window > $O/${w}_one$one.json 2> $O/$w.err || { echo FAIL $w $one; tail -20 $O/$w.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/${w}_one$one.json').read().strip().splitlines()[-1]); b=d['block']
print('$w onelaunch $one', round(d['value']), 'la', b['lookahead'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), d['pivot_log_vs_oracle'])"
done; done
