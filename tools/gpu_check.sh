#!/bin/bash
# One GPU verification pass (run through gpurun from the repo root):
#   tools/gpu_check.sh <tag> [pytest -k expression]
# Writes under gpurun_out/<tag>/: the -m gpu test log, smoke(), the default
# bench line (driver protocol: --steps 20 --warmup 5) and a rocprofv3
# kernel-trace profile of that same command (tools/gpu_profile.sh).
# Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R=$(pwd)
TAG=${1:-check}
K=${2:-}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
rocm-smi --showproductname > $OUT/gpu.txt 2>&1 || true
KARG=()
[ -n "$K" ] && KARG=(-k "$K")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    "${KARG[@]}" > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 1; }
tail -3 $OUT/gpu_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 \
    || { cat $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
timeout -k 10 300 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err \
    || { cat $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
echo "check $TAG done"
