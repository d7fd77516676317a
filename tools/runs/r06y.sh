#!/bin/bash
# r06y: chain phase stamps (tools/chain_stamps.py) at C3 (grouped ring, and the LEAN ring) and c3r8
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06y; mkdir -p $O
timeout -k 10 300 python3 tools/chain_stamps.py > $O/c3_grouped.json || exit 1
DLP_RATIO_ROWS=0 timeout -k 10 300 python3 tools/chain_stamps.py > $O/c3_lean.json || exit 1
timeout -k 10 300 python3 tools/chain_stamps.py --workload c3r8 > $O/c3r8.json || exit 1
for f in c3_grouped c3_lean c3r8; do python3 -c "
import json; d=json.load(open('$O/$f.json')); print('$f', d['bench_value'], d['pass_ms']); [print('   %-58s %6.1f' % (k, v)) for k, v in d['median_us'].items()]"; done
echo done
