#!/bin/bash
# r06s: chainlab, workgroup shapes the product can take without changing the exchange's candidate
# slots (rows per ratio workgroup = the session's ratio threads), and 512-column pivot-row workgroups.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r06s
mkdir -p $OUT build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o build/chainlab tools/chainlab.hip || exit 1
: > $OUT/lab.jsonl
run() { timeout -k 5 30 "$@" >> $OUT/lab.jsonl || { echo "FAIL $* rc=$?"; exit 1; }; }
for J in 64 127; do
  for spec in "4096 128 g16x16x2 512" "4096 128 g16x16x2 256" "4096 128 g16x16x2 128" "4096 128 g32x16x4 256" "4096 128 g32x16x4 128" \
              "4096 128 g16x8x1 512" "4096 128 g64x16x4 128" "4096 128 ring 128" \
              "8192 128 g32x16x4 256" "8192 128 g32x16x4 128" "8192 128 g16x16x2 512" "8192 128 g64x16x4 128" "8192 128 ring 128" \
              "16384 64 g64x16x4 256" "16384 64 g32x16x4 512" "16384 64 g32x16x4 256" "16384 64 ring 256" \
              "32768 64 g64x16x4 256" "32768 64 ring 256"; do
    set -- $spec
    LAB_THREADS=$4 run build/chainlab ratio $3 $1 $J $2 16
  done
  for cus in 128 64; do
    for v in fat ringg q64x16x4t512 q64x12x4t512 ring1; do
      run build/chainlab prow $v 32768 $J $cus 8
    done
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r06s/lab.jsonl"):
    r=json.loads(l)
    print(f"{r['kernel']:5s} {r['variant']:13s} t={r.get('threads',0):4d} n={r['n']:6d} steps={r['steps']:3d} cus={r['cus']:3d} {r['us_per_launch']:7.2f} us bad={r['mismatches']}")
PY
echo done
