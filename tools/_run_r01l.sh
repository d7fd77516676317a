#!/bin/bash
# Round-1 evidence with pass form 4 at K = 32: full GPU suite, smoke, default
# bench (CPU baseline included), C2 bench, rocprof stats + HBM PMC passes.
set -o pipefail
O=gpurun_out/r01l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && \
timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err && \
bash tools/gpu_profile.sh r01l_prof && \
echo "r01l done"
