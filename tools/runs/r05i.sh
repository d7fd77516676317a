#!/bin/bash
# r05i (lab): the VALU-DPP ring pass (f4r) and the MFMA pass (mpass4) concurrently on every CU, each on a share of
# the columns (C3, out of place, ld 65,664)
set -o pipefail
O=gpurun_out/r05i; mkdir -p $O
export LAB_LD=65664 LAB_OOP=1
timeout -k 10 300 tools/lab5/passlab 32768 65537 5 hetero > $O/lab_hetero.txt 2>&1 || { tail -20 $O/lab_hetero.txt; exit 1; }
cat $O/lab_hetero.txt
