#!/bin/bash
# Iteration run: deferred + eager parity tests, bench (default and per-phase timing), kernel stats.
#   bash tools/_run_iter.sh <tag>
set -o pipefail
TAG=${1:-iter}
O=gpurun_out/$TAG
mkdir -p $O
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_parity.py tests/test_gpu_general.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline --timing 2 > $O/bench_t2.json 2> $O/bench_t2.err && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline > $R/$O/trace_bench.json 2> $R/$O/trace.err) && \
echo "iter $TAG done"
