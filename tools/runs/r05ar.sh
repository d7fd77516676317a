#!/bin/bash
# r05ar: same-box A/B of the chain-kernel load changes (r05ao-r05aq: loads without per-load branches, the pivot-row
# replay's first chunk early, the state in one round trip) against the build before them; alternating C2 and c3r8
set -o pipefail
O=gpurun_out/r05ar; mkdir -p $O
run() {  # tag lib args
cp tools/ab/libdlp_$2.so distributedlpsolver_amd/libdlp.so || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window $3 > $O/$1.json 2> $O/$1.err || { echo FAIL $1; tail -20 $O/$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', round(d['value']))"
}
for r in a b c; do
run c2new$r new "--workload c2" && run c2prev$r prev "--workload c2" && run r8new$r new "--workload c3r8" && run r8prev$r prev "--workload c3r8" || exit 1
done
cp tools/ab/libdlp_new.so distributedlpsolver_amd/libdlp.so
