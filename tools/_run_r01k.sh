#!/bin/bash
# Round-1 evidence after the small-tableau auto policy (eager under 32 MiB): full GPU suite, smoke,
# default bench (CPU baseline included), secondary measurements (C1 / C4 / C5 / f1).
set -o pipefail
O=gpurun_out/r01k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && \
timeout -k 10 500 python -u tools/bench_extra.py --out $O/extra.json > $O/extra.log 2>&1 && \
echo "r01k done"
