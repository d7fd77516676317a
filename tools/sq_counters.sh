#!/bin/bash
# SQ wave-state counters of one kernel (run through gpurun from the repo root):
#   tools/sq_counters.sh <tag> <kernel-substring> [bench args...]
# One rocprofv3 --pmc pass of 8 SQ counters (the SQ block's slot count,
# MI355X_MICROARCH.md §rocprofv3 PMC slots) over a short bench.py run, then
# tools/sq_summary.py <dir> <kernel-substring>.
set -o pipefail
R=$(pwd)
TAG=$1; SUB=$2; shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM --output-format csv -d $OUT/sq -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-pivot-window "$@" > $OUT/sq_bench.json 2> $OUT/sq.err || exit $?
cd $R && python3 tools/sq_summary.py $OUT/sq "$SUB" > $OUT/sq_summary.json && cat $OUT/sq_summary.json
