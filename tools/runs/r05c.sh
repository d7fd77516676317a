#!/bin/bash
# r05c (lab): tools/passlab.hip round-5 variants, out of place at ld 65,664 as the product's lookahead pass:
# band counts vs the 768 pass slots; the interleaved persistent ring pass on exactly 256 tiles; MFMA at 3-4 waves/SIMD
set -o pipefail
O=gpurun_out/r05c; mkdir -p $O
export LAB_LD=65664 LAB_OOP=1
timeout -k 10 240 tools/lab5/passlab 32768 65537 5 "r5 f4r rb" > $O/lab_rb.txt 2>&1 || { tail -20 $O/lab_rb.txt; exit 1; }
cat $O/lab_rb.txt
timeout -k 10 240 tools/lab5/passlab 32768 65536 5 "r5 f4r" > $O/lab_il.txt 2>&1 || { tail -20 $O/lab_il.txt; exit 1; }
cat $O/lab_il.txt
timeout -k 10 240 tools/lab5/passlab 32768 65537 5 "r5 mpass4" > $O/lab_mfma.txt 2>&1 || { tail -20 $O/lab_mfma.txt; exit 1; }
cat $O/lab_mfma.txt
