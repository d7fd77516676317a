#!/bin/bash
# r05w: why C3 over 4 processes on one GPU stalled (r05v): 4 rank processes of smaller LPs and of C3 with the CU split
# off / lookahead off / 3 processes; every run bounded by its exchange timeout (30 s)
set -o pipefail
O=gpurun_out/r05w; mkdir -p $O
run() {  # tag args...
timeout -k 10 240 python -u tools/rank_procs.py "${@:2}" > $O/$1.json 2> $O/$1.err || { echo FAIL $1; tail -5 $O/$1.err; }
python3 -c "
import json
d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1])
print('$1', [(r.get('run'), round(r.get('seconds',-1),2), r.get('run_error','')[:80], r.get('error','')[:80], r.get('config')) for r in d['ranks']])" || true
}
run p4small 8192 57344 34 4 136
run p4c3nomask 32768 32768 3 4 136 DLP_CHAIN_CUS=0
run p4c3nola 32768 32768 3 4 136 LOOKAHEAD=0
run p3c3 32768 32768 3 3 136
run p4c3 32768 32768 3 4 136
