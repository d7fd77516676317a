#!/bin/bash
# r06t: the grouped-ring selection kernel (ratio_ring_kernel) in the product: parity (the lookahead,
# large and rank-process suites against the oracle's digests), then alternating A/B against the
# LEAN ring (DLP_RATIO_ROWS=0) at C3 and the rank geometries.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r06t
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_large.py tests/test_gpu_knobs.py tests/test_gpu_ranks.py > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
B="python -u bench.py --no-cpu-baseline --no-pivot-window --no-eager-window --steps 20 --warmup 5"
for w in c3r8 c3r4 c3 c3r2; do
  for rep in 1 2; do
    for rr in default 0; do
      if [ $rr = default ]; then E=""; else E="DLP_RATIO_ROWS=$rr"; fi
      env $E timeout -k 10 240 $B --workload $w > $OUT/${w}_rows${rr}_$rep.json 2> $OUT/${w}_rows${rr}_$rep.err || { echo "bench $w $rr rc=$?"; exit 1; }
      python3 -c "import json,sys; d=json.load(open('$OUT/${w}_rows${rr}_$rep.json')); print('$w rows=$rr rep=$rep', round(d['value']), 'pivots/s', 'block', d['ms_per_step'])"
    done
  done
done
for rr in 16 32; do
  DLP_RATIO_ROWS=$rr timeout -k 10 240 $B --workload c3r8 > $OUT/c3r8_rows${rr}_x.json 2> $OUT/c3r8_rows${rr}_x.err || { echo "bench c3r8 $rr rc=$?"; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/c3r8_rows${rr}_x.json')); print('c3r8 rows=$rr', round(d['value']), 'pivots/s')"
done
echo done
