#!/bin/bash
# Deferred ratio kernel at 128 threads per workgroup (257 workgroups at C3): parity + bench + kernel stats.
set -o pipefail
O=gpurun_out/it9
mkdir -p $O
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_gpu_defer.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 && \
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline > $R/$O/trace_bench.json 2> $R/$O/trace.err) && \
echo "it9 done"
