#!/bin/bash
# lab10: dependent-load latency (MALL-resident table) beside an nt stream, by stream workgroups
set -o pipefail
mkdir -p gpurun_out/lab tools/bin; O=gpurun_out/lab/lab10.txt; : > $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/mall_probe tools/mall_probe.hip || exit 1
for w in 0 2048 1024 768 512 256 128; do
timeout -k 10 60 tools/bin/mall_probe 48 8192 $w lat >> $O 2>&1 || { tail $O; exit 1; }
done
cat $O
