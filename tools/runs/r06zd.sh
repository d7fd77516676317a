#!/bin/bash
# r06zd: c3r8 chain phases with the LEAN pivot-row kernel (it carries the stamps): where the pivot-row launch goes
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06zd; mkdir -p $O
DLP_FAT_PROW=0 timeout -k 10 300 python3 tools/chain_stamps.py --workload c3r8 > $O/c3r8_lean_prow.json || exit 1
DLP_FAT_PROW=0 timeout -k 10 300 python3 tools/chain_stamps.py --workload c3r2 > $O/c3r2_lean_prow.json || exit 1
for f in c3r8_lean_prow c3r2_lean_prow; do python3 -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['bench_value'], d['pass_ms']); [print('   %-58s %6.1f' % (k, v)) for k, v in d['median_us'].items()]"; done
echo done
