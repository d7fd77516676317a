#!/bin/bash
# C5 (4,096 x 64 x 128 LPs) on one MI355X: kernel-trace stats and LDS / wave-state counters of
# batched_solve_kernel (run through gpurun from the repo root): tools/c5_profile.sh <tag>
set -o pipefail
R=$(pwd); TAG=${1:-c5}; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 120 python3 tools/c5_run.py 64 128 5 > $OUT/c5_run.json || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 $R/tools/c5_run.py 64 128 3 > $OUT/trace_run.json 2> $OUT/trace.err || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
    SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU --output-format csv -d $OUT/lds -o run -- \
    python3 $R/tools/c5_run.py 64 128 1 > $OUT/lds_run.json 2> $OUT/lds.err || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH --output-format csv -d $OUT/state -o run -- \
    python3 $R/tools/c5_run.py 64 128 1 > $OUT/state_run.json 2> $OUT/state.err || exit 1
cd $R && python3 tools/sq_summary.py $OUT/lds batched_solve > $OUT/lds_summary.json && \
    python3 tools/sq_summary.py $OUT/state batched_solve > $OUT/state_summary.json; cat $OUT/c5_run.json $OUT/lds_summary.json $OUT/state_summary.json
