#!/bin/bash
# lab8: MALL residency of a 48 MB table across a 2 GB stream, per stream cache policy
set -o pipefail
mkdir -p gpurun_out/lab tools/bin
hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bin/mall_probe tools/mall_probe.hip || exit 1
timeout -k 10 120 tools/bin/mall_probe 48 2048 > gpurun_out/lab/lab8.txt 2>&1 || { tail gpurun_out/lab/lab8.txt; exit 1; }
timeout -k 10 120 tools/bin/mall_probe 48 256 >> gpurun_out/lab/lab8.txt 2>&1 || { tail gpurun_out/lab/lab8.txt; exit 1; }
cat gpurun_out/lab/lab8.txt
