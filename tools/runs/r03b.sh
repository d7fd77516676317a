#!/bin/bash
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03b; mkdir -p $OUT
timeout -k 10 420 python -u -m pytest tests/test_gpu_peer.py -v --timeout 120 --timeout-method thread \
   -k "not c3_row_partition" > $OUT/peer_tests.txt 2>&1; rc=$?
tail -25 $OUT/peer_tests.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1) || true
for S in state insts; do
  SQ_SET=$S bash tools/sq_counters.sh r03b_la pass_d_kernel --steps 6 --warmup 2 || exit 1
  for k in ratio_lean_kernel prow_defer_kernel; do python3 tools/sq_summary.py gpurun_out/r03b_la/sq_$S $k > gpurun_out/r03b_la/sq_${S}_$k.json || true; done
done
for S in state insts; do
  SQ_SET=$S bash tools/sq_counters.sh r03b_nola pass_d_kernel --steps 6 --warmup 2 --lookahead 0 || exit 1
  for k in ratio_defer_kernel prow_defer_kernel; do python3 tools/sq_summary.py gpurun_out/r03b_nola/sq_$S $k > gpurun_out/r03b_nola/sq_${S}_$k.json || true; done
done
timeout -k 10 300 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
