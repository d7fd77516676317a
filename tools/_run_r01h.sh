#!/bin/bash
# Round-1 re-verification after the container was re-created: full GPU suite, smoke,
# default bench (with CPU baseline), rocprof stats + HBM PMC passes of the same command.
set -o pipefail
O=gpurun_out/r01h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && \
bash tools/gpu_profile.sh r01h_prof && \
echo "r01h done"
