#!/bin/bash
# r06q: chain replay loops in isolation (tools/chainlab.hip): ring / grouped ring / 16-row waves /
# registers for the ratio replay, register / LDS-ring variants for the pivot-row replay, at the c3r8
# (4,096 rows, chain on 128 CUs) and C3 (32,768 rows, 64 CUs) geometries, warm and cold inputs.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r06q
mkdir -p $OUT build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o build/chainlab tools/chainlab.hip || exit 1
: > $OUT/lab.jsonl
for n_cus in "4096 128" "32768 64"; do
  set -- $n_cus
  for J in 64 127; do
    for cp in 1 16; do
      for v in ring ringg ringg2 r16 reg; do
        timeout -k 5 30 build/chainlab ratio $v $1 $J $2 $cp >> $OUT/lab.jsonl || { echo "FAIL ratio $v $1 $J $cp rc=$?"; exit 1; }
      done
    done
  done
done
for cus in 128 64; do
  for S in 64 127; do
    for cp in 1 8; do
      for v in fat fat1 ringg ring8 ring1; do
        timeout -k 5 30 build/chainlab prow $v 32768 $S $cus $cp >> $OUT/lab.jsonl || { echo "FAIL prow $v $S $cp rc=$?"; exit 1; }
      done
    done
  done
done
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/r06q/lab.jsonl")]
for r in rows:
    print(f"{r['kernel']:5s} {r['variant']:7s} n={r['n']:6d} steps={r['steps']:3d} cus={r['cus']:3d} copies={r['copies']:2d} {r['us_per_launch']:7.2f} us (empty {r['empty_us']:.2f}) bad={r['mismatches']}")
PY
echo done
