#!/bin/bash
# r06zc: condensed C3 with the MFMA pass (form 22) against the LDS-ring DPP pass (form 23), in situ and alone
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zc; mkdir -p $O
run() {  # tag args...
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'pass', round(r['launch_ms'],3), 'frac', round(r['frac'],3), 'fp64', round(r['fp64_frac'],3), 'fp64_cus', r.get('fp64_frac_of_pass_cus') and round(r['fp64_frac_of_pass_cus'],3), 'form', d['geometry'].get('form'))"
}
for r in a b; do
run f23_$r || exit 1
run f22_$r --form 22 || exit 1
run f23la0_$r --lookahead 0 || exit 1
run f22la0_$r --form 22 --lookahead 0 || exit 1
done
echo done
