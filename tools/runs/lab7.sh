#!/bin/bash
# lab7: out-of-place copy in form 21's shape, wide workgroups x band heights
set -o pipefail
mkdir -p gpurun_out/lab tools/bin; O=gpurun_out/lab/lab7.txt; : > $O
hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/bin/passlab tools/passlab.hip || exit 1
LAB_LD=65664 LAB_OOP=1 timeout -k 10 300 tools/bin/passlab 32768 65537 5 copyw >> $O 2>&1 || { tail $O; exit 1; }
cat $O
