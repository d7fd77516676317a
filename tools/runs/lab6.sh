#!/bin/bash
mkdir -p gpurun_out/lab; O=gpurun_out/lab/lab6.txt; : > $O
for LD in 66048 65552 65600 65664 66560 67072; do
  echo "== ld $LD" >> $O
  LAB_LD=$LD LAB_OOP=1 timeout -k 10 120 tools/bin/passlab 32768 65537 3 "f4r K64" >> $O 2>&1 || exit 1
done
timeout -k 10 60 python3 tools/c1_overhead.py > gpurun_out/lab/c1_overhead.json 2>gpurun_out/lab/c1_overhead.err || exit 1
grep -v "^check" $O; cat gpurun_out/lab/c1_overhead.json
