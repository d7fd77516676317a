#!/bin/bash
# r04al: C3's form-21 pass alone (no lookahead, in place) vs in situ beside the chain (the default)
set -o pipefail
O=gpurun_out/r04al; mkdir -p $O
run() {  # tag args...
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "${@:2}" > $O/c3_$1.json 2> $O/c3.err || { echo FAIL $1; tail -20 $O/c3.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_$1.json').read().strip().splitlines()[-1]); b=d['block']; r=d['roofline']
print('c3 $1', round(d['value']), 'form', d['geometry']['form'], 'la', b['lookahead'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'frac', round(r['frac'],4))"
}
for k in 1 2; do
run default_$k && run f21_alone_$k --lookahead 0 --form 21 && run f23_alone_$k --lookahead 0 || exit 1
done
