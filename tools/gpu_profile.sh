#!/bin/bash
# Profile the bench workload on one MI355X (run through gpurun from the repo root).
#   tools/gpu_profile.sh <tag> [bench args...]
# Writes under gpurun_out/<tag>/: kernel-trace stats, FETCH_SIZE and WRITE_SIZE
# passes (separate, as MI355X_MICROARCH.md's rocprofv3 section requires).
set -o pipefail
R=$(pwd)
TAG=${1:-prof}; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline "$@" > $OUT/trace_bench.json 2> $OUT/trace.err || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 32 --warmup 16 "$@" > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- \
    python3 $R/bench.py --no-cpu-baseline --steps 32 --warmup 16 "$@" > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit $?
echo "profile $TAG done"
