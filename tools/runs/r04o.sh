#!/bin/bash
# r04o: why the chain-stamp runs are slow at c3r8 (short windows vs stamps); bench.py's guarded run
set -o pipefail
O=gpurun_out/r04o; mkdir -p $O
run() {  # tag args...
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window "${@:2}" > $O/$1.json 2> $O/$1.err || { echo FAIL $1; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'steps', d['steps'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), d.get('exchange'), d.get('exchange_fallback_reason'))"
}
run c3r8_s3w2 --workload c3r8 --no-pivot-window --steps 3 --warmup 2 && run c3r8_s20 --workload c3r8 --no-pivot-window
DLP_CHAIN_STAMPS=$PWD/$O/st.bin run c3r8_stamps_s20 --workload c3r8 --no-pivot-window
DLP_CHAIN_STAMPS=$PWD/$O/st.bin run c3r8_stamps_s3w2 --workload c3r8 --no-pivot-window --steps 3 --warmup 2
run c3_default
