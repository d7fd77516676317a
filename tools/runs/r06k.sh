#!/bin/bash
# r06k: block size at the condensed rank geometries and C3 under lookahead (K = 16 / 32 forced vs the K = 64
# default), then the knob tests (DLP_CONDENSED=0 equivalence)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06k; mkdir -p $O
run() {  # tag workload args...
  tag=$1; w=$2; shift 2
  timeout -k 10 300 python3 bench.py --workload $w --no-cpu-baseline --no-eager-window --no-pivot-window "$@" > $O/$tag.json 2> $O/$tag.err || { echo FAIL $tag; tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); r=d['roofline']; b=d['block']
print('$tag', round(d['value']), 'block', round(b['ms'],3), 'K', d['K'], 'pass', round(r['launch_ms'],3), 'form', d['geometry']['form'], 'cus', b.get('chain_cus'), 'la', b['lookahead'])"
}
for w in c3r8 c3r4 c3r2; do
run ${w}_k64 $w || exit 1
run ${w}_k32 $w --defer 32 --lookahead 1 || exit 1
run ${w}_k16 $w --defer 16 --lookahead 1 --steps 40 || exit 1
done
run c3_k64 c3 || exit 1
run c3_k32 c3 --defer 32 --lookahead 1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_knobs.py -v --timeout 300 --timeout-method thread > $O/knobs.log 2>&1 || { grep -E "FAILED|^E " $O/knobs.log | head; exit 1; }
tail -1 $O/knobs.log
