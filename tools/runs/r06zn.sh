#!/bin/bash
# r06zn: chainlab, the register pivot-row replay with 2 x 16 / 24 / 32 rows in flight per wave (the pivot-row
# launch holds one workgroup per CU at the rank geometries, so registers are free)
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r06zn
mkdir -p $OUT build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o build/chainlab tools/chainlab.hip || exit 1
: > $OUT/lab.jsonl
for S in 32 48 64 96 127; do
  for v in fat fat24 fat32; do
    timeout -k 5 30 build/chainlab prow $v 32768 $S 96 8 >> $OUT/lab.jsonl || { echo "FAIL $v $S"; exit 1; }
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r06zn/lab.jsonl"):
    r=json.loads(l); print(r['variant'], r['steps'], r['us_per_launch'], 'bad', r['mismatches'])
PY
