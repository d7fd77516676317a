#!/bin/bash
mkdir -p gpurun_out/lab; O=gpurun_out/lab/lab5.txt; : > $O
for v in "f4r K64 U4 D3 w3" "f4q K64 V1U2 w3 rb768"; do
  timeout -k 10 100 tools/bin/passlab 32768 65537 5 "$v" >> $O 2>&1 || exit 1
  LAB_OOP=1 timeout -k 10 100 tools/bin/passlab 32768 65537 5 "$v" >> $O 2>&1 || exit 1
done
timeout -k 10 200 tools/bin/passlab 32768 65537 3 copy >> $O 2>&1 || exit 1
grep -v "^check" $O
