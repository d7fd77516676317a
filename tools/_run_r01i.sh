#!/bin/bash
# Round-1 evidence after the ratio/prow latency changes: full GPU suite, smoke, default bench
# (CPU baseline included), rocprof stats + HBM PMC passes; then a K = 32 pass-form sweep.
set -o pipefail
O=gpurun_out/r01i
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && \
timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err && \
bash tools/gpu_profile.sh r01i_prof && \
timeout -k 10 400 python tools/tune_defer.py --ks 32 --forms 3,5 --rbs 128,256 --occs 0,3 --rounds 3 > $O/tune_k32_forms35.txt 2>&1 && \
echo "r01i done"
