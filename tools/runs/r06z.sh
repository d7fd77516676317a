#!/bin/bash
# r06z: per-workgroup stamps of one grouped-ring selection per block (C3, c3r2): where the ratio
# launch's last workgroup loses its time
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06z; mkdir -p $O
timeout -k 10 300 python3 tools/chain_stamps.py > $O/c3.json || exit 1
timeout -k 10 300 python3 tools/chain_stamps.py --workload c3r2 > $O/c3r2.json || exit 1
DLP_RATIO_ROWS=32 timeout -k 10 300 python3 tools/chain_stamps.py --workload c3r8 > $O/c3r8.json || exit 1
for f in c3 c3r2 c3r8; do python3 -c "
import json; d=json.load(open('$O/$f.json')); print('$f', json.dumps(d['workgroups'], indent=1))"; done
echo done
