#!/bin/bash
# r05n: C3 pass workgroups held to 2 per CU (DLP_PASS_LDS) so the chain beside them shares each SIMD with 2 pass
# waves instead of 3; the LDS-ring pass (form 23) with deeper rings to keep its stream; alternating
set -o pipefail
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 600 python -u -m pytest "tests/test_gpu_knobs.py::test_form23_ring_depth" tests/test_gpu_knobs.py::test_pass_lds_cap -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo FAIL tests; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # tag args env...
timeout -k 10 300 env "${@:3}" python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window $2 > $O/c3_$1.json 2> $O/c3_$1.err || { echo FAIL $1; tail -20 $O/c3_$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'form', d['geometry']['form'])"
}
for r in a b; do
run def$r "" X=0 && run f23$r "--form 23" X=0 && run f23l56$r "--form 23" DLP_PASS_LDS=57344 && run f23d6l56$r "--form 23" DLP_PASS_LDS=57344 DLP_Q_DEPTH=6 && run f23d8$r "--form 23" DLP_Q_DEPTH=8 && run f21l56$r "" DLP_PASS_LDS=57344 && run c32$r "" DLP_CHAIN_CUS=32 || exit 1
done
