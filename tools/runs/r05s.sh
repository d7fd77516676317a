#!/bin/bash
# r05s: C3 with the ratio launch on 128- and 64-lane workgroups (DLP_RATIO_THREADS: 256 or 512 workgroups,
# the chain's waves on every CU instead of every other one) beside the form-21 and form-23 passes; alternating
set -o pipefail
O=gpurun_out/r05s; mkdir -p $O
run() {  # tag args env...
timeout -k 10 300 env "${@:3}" python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window $2 > $O/c3_$1.json 2> $O/c3_$1.err || { echo FAIL $1; tail -20 $O/c3_$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'form', d['geometry']['form'])"
}
for r in a b; do
run def$r "" X=0 && run t128$r "" DLP_RATIO_THREADS=128 && run t64$r "" DLP_RATIO_THREADS=64 \
 && run f23$r "--form 23" X=0 && run f23t128$r "--form 23" DLP_RATIO_THREADS=128 && run f23t64$r "--form 23" DLP_RATIO_THREADS=64 || exit 1
done
timeout -k 10 300 env DLP_RATIO_THREADS=64 python -u tools/chain_stamps.py --form 23 > $O/stamps_f23t64.json 2> $O/stamps_f23t64.err || { echo FAIL stamps; tail -20 $O/stamps_f23t64.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/stamps_f23t64.json')); print(d['bench_value'], {k: round(v,1) for k,v in d['median_us'].items()})"
