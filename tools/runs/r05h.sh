#!/bin/bash
# r05h: the MID chain kernels (register replay, <= 104 VGPRs) beside the MFMA pass (form 22): lookahead tests
# with form 22, then C3 alternating form 21 / form 22 + MID / form 22 + LEAN (DLP_MID_CHAIN=0); c3r8 / c3r4 form 22
set -o pipefail
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_lookahead.py "tests/test_gpu_defer.py::test_pass_form21_dpp_full_blocks" "tests/test_gpu_peer.py::test_peer_exchange_lookahead_k64" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo FAIL tests; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
run() {  # workload tag args env...
timeout -k 10 300 env "${@:4}" python -u bench.py --workload $1 --no-cpu-baseline --no-eager-window --no-pivot-window $3 > $O/$1_$2.json 2> $O/$1_$2.err || { echo FAIL $1 $2; tail -20 $O/$1_$2.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1_$2.json').read().strip().splitlines()[-1]); b=d['block']
print('$1 $2', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'frac', round(d['roofline']['frac'],4), 'form', d['geometry']['form'], 'cus', b['chain_cus'])"
}
for r in a b; do
run c3 f21$r "" X=0 && run c3 f22mid$r "--form 22" X=0 && run c3 f22lean$r "--form 22" DLP_MID_CHAIN=0 || exit 1
done
for r in a b; do
run c3r8 def$r "" X=0 && run c3r8 f22$r "--form 22" X=0 && run c3r8 cus160$r "" DLP_CHAIN_CUS=160 && run c3r8 cus192$r "" DLP_CHAIN_CUS=192 && run c3r8 mid$r "" DLP_MID_CHAIN=1 && run c3r4 def$r "" X=0 && run c3r4 f22$r "--form 22" X=0 || exit 1
done
