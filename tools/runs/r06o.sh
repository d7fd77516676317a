#!/bin/bash
# r06o: C5 (4,096 x 64 x 128 batched solve) SQ counters for a hardware-anchored bound: wave states, instruction
# counts, LDS activity (three --pmc passes, each its own run)
set -o pipefail
for set in state insts lds; do
  SQ_SET=$set timeout -k 10 200 bash tools/sq_counters.sh r06o batched_reg_kernel --workload c5 --steps 3 --warmup 1 > /dev/null 2> gpurun_out/r06o_$set.err || { echo FAIL $set; tail -5 gpurun_out/r06o_$set.err; cat gpurun_out/r06o/sq_$set.err 2>/dev/null | tail -5; exit 1; }
  cat gpurun_out/r06o/sq_${set}_summary.json
done
