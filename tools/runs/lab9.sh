#!/bin/bash
# lab9: a 48 MB table's read rate while an nt stream runs beside it, by stream workgroups
set -o pipefail
mkdir -p gpurun_out/lab tools/bin; O=gpurun_out/lab/lab9.txt; : > $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/mall_probe tools/mall_probe.hip || exit 1
for w in 0 2048 1024 512 256; do
timeout -k 10 60 tools/bin/mall_probe 48 8192 $w >> $O 2>&1 || { tail $O; exit 1; }
done
cat $O
