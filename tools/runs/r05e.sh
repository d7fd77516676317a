#!/bin/bash
# r05e: form 22 (MFMA pass, 128-column workgroups, 3 waves/SIMD) now publishes its bands under lookahead:
# the lookahead + form tests, then C3 alternating: form 21 (default) vs form 22, and 128-lane ratio workgroups
set -o pipefail
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_lookahead.py "tests/test_gpu_defer.py::test_pass_form21_dpp_full_blocks" "tests/test_gpu_defer.py::test_pass_form21_sparse_and_degenerate" tests/test_gpu_ranks.py "tests/test_gpu_knobs.py::test_lookahead_chain_knobs" tests/test_gpu_knobs.py::test_ratio_threads_without_lookahead -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo FAIL tests; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
run() {  # tag args/env...
timeout -k 10 300 env "${@:3}" python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window $2 > $O/c3_$1.json 2> $O/c3_$1.err || { echo FAIL $1; tail -20 $O/c3_$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'frac', round(d['roofline']['frac'],4), 'form', d['geometry']['form'], 'la', b['lookahead'])"
}
run f21a "" X=0 && run f22a "--form 22" X=0 && run r128a "" DLP_RATIO_THREADS=128 && run f22r128a "--form 22" DLP_RATIO_THREADS=128 && \
run f21b "" X=0 && run f22b "--form 22" X=0 && run r128b "" DLP_RATIO_THREADS=128 && run f22r128b "--form 22" DLP_RATIO_THREADS=128
