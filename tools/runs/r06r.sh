#!/bin/bash
# r06r: chainlab, second sweep: rows per wave x DMAs in flight x DMAs per wait (ratio), columns per
# wave (pivot row), at the c3r8 / c3r4 / C3 geometries; cold inputs (copies 16 / 8).
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r06r
mkdir -p $OUT build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o build/chainlab tools/chainlab.hip || exit 1
: > $OUT/lab.jsonl
run() { timeout -k 5 30 "$@" >> $OUT/lab.jsonl || { echo "FAIL $* rc=$?"; exit 1; }; }
for n_cus in "4096 128" "8192 128" "32768 64"; do
  set -- $n_cus
  for J in 64 127; do
    for v in ring ringg g64x16x4 g64x24x8 g64x32x8 g32x16x2 g32x16x4 g16x8x1 g16x16x2; do
      run build/chainlab ratio $v $1 $J $2 16
    done
    LAB_THREADS=64 run build/chainlab ratio g64x16x4 $1 $J $2 16
    LAB_THREADS=64 run build/chainlab ratio g32x16x4 $1 $J $2 16
  done
done
for cus in 128 64; do
  for S in 64 127; do
    for v in fat ringg ringg128 ring1 q64x16x8 q64x24x8 q32x16x4 q32x16x4t128; do
      run build/chainlab prow $v 32768 $S $cus 8
    done
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r06r/lab.jsonl"):
    r=json.loads(l)
    print(f"{r['kernel']:5s} {r['variant']:13s} n={r['n']:6d} steps={r['steps']:3d} cus={r['cus']:3d} {r['us_per_launch']:7.2f} us bad={r['mismatches']}")
PY
echo done
