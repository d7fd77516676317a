#!/bin/bash
# r04m: c3r8 with the lookahead pass on a CU-masked stream (DLP_PASS_CUS, experiment)
set -o pipefail
O=gpurun_out/r04m; mkdir -p $O
run() {  # tag env...
env "${@:2}" timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline --no-eager-window --no-pivot-window > $O/${W}_$1.json 2> $O/$W.err || { echo FAIL $1; tail -20 $O/$W.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/${W}_$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$W $1', round(d['value']), 'la', b['lookahead'], 'form', d['geometry']['form'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3))"
}
W=c3r8
run base X=0 && run prio DLP_CHAIN_SETPRIO=1 && run ring16 DLP_RING_DEPTH=16 && run ring32 DLP_RING_DEPTH=32 && run low128 DLP_PASS_CUS=128 && run spread128 DLP_PASS_CUS=128 DLP_PASS_CUS_MODE=spread && run low192 DLP_PASS_CUS=192 && run spread192 DLP_PASS_CUS=192 DLP_PASS_CUS_MODE=spread && run spread64 DLP_PASS_CUS=64 DLP_PASS_CUS_MODE=spread && run spread96 DLP_PASS_CUS=96 DLP_PASS_CUS_MODE=spread
W=c3r4
run base X=0 && run prio DLP_CHAIN_SETPRIO=1 && run ring16 DLP_RING_DEPTH=16 && run ring32 DLP_RING_DEPTH=32 && run spread128 DLP_PASS_CUS=128 DLP_PASS_CUS_MODE=spread && run spread192 DLP_PASS_CUS=192 DLP_PASS_CUS_MODE=spread
W=c3
run base X=0 && run prio DLP_CHAIN_SETPRIO=1
DLP_TRACE_CREATE=1 timeout -k 10 120 python -u tools/c1_overhead.py > $O/c1_overhead.json 2> $O/c1_stages.txt || { echo C1_FAIL; tail $O/c1_stages.txt; exit 1; }
tail -24 $O/c1_stages.txt
