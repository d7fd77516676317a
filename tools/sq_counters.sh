#!/bin/bash
# SQ counters of a short bench.py run (run through gpurun from the repo root):
#   SQ_SET=state|insts tools/sq_counters.sh <tag> <kernel-substring> [bench args...]
# One rocprofv3 --pmc pass of at most 8 SQ counters (the SQ block's slot count,
# MI355X_MICROARCH.md §rocprofv3 PMC slots), then tools/sq_summary.py <dir> <kernel>.
#   state: wave states (parked / issue-stalled / active, VALU-active cycles)
#   insts: instruction counts per launch (VALU, VMEM reads / writes, SALU, SMEM, LDS)
#   lds:   LDS activity and bank conflicts beside the VALU-active cycles
set -o pipefail
R=$(pwd)
TAG=$1; SUB=$2; shift 2
SET=${SQ_SET:-state}
case $SET in
  state) CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM";;
  insts) CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS";;
  lds) CTRS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY";;
  *) echo "unknown SQ_SET $SET"; exit 2;;
esac
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/sq_$SET -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-pivot-window --no-eager-window "$@" \
    > $OUT/sq_${SET}_bench.json 2> $OUT/sq_$SET.err || exit $?
cd $R && python3 tools/sq_summary.py $OUT/sq_$SET "$SUB" > $OUT/sq_${SET}_summary.json && cat $OUT/sq_${SET}_summary.json
