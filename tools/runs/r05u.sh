#!/bin/bash
# r05u: chain phase stamps at c3r8 (chain on 128 CUs of its own; diagnostics, never a timed figure), with the register
# pivot-row kernel (default, unstamped) and with the LEAN one (stamped)
set -o pipefail
O=gpurun_out/r05u; mkdir -p $O
st() {  # tag env... -- args
timeout -k 10 300 env "${@:2}" python -u tools/chain_stamps.py --workload c3r8 > $O/stamps_$1.json 2> $O/stamps_$1.err || { echo FAIL $1; tail -20 $O/stamps_$1.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/stamps_$1.json')); print('$1', round(d['bench_value']), {k: round(v,1) for k,v in d['median_us'].items()})"
}
st def X=0 && st leanprow DLP_FAT_PROW=0
