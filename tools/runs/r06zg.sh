#!/bin/bash
# r06zg: C3 selection ring with 12 DMAs in flight (3 workgroups per chain CU: all 129 resident) vs 16
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zg; mkdir -p $O
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3))"
}
for r in a b c; do
run rp16_$r || exit 1
DLP_RATIO_RP=12 run rp12_$r || exit 1
done
DLP_RATIO_RP=12 timeout -k 10 300 python3 tools/chain_stamps.py > $O/stamps_rp12.json || exit 1
python3 -c "
import json; d=json.load(open('$O/stamps_rp12.json')); print('rp12 stamps', d['bench_value']); [print('   %-58s %6.1f' % (k, v)) for k, v in d['median_us'].items()]; w=d['workgroups']; print(w and {k: w[k] for k in ('start_us','ticket_us')})"
echo done
