#!/bin/bash
# r04g: C3 with the lookahead chain on CUs of its own (DLP_CHAIN_CUS, CU-masked streams)
set -o pipefail
O=gpurun_out/r04g; mkdir -p $O
for c in 0 16 32 0 16 8; do
DLP_CHAIN_CUS=$c timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/c3_cus$c.json 2> $O/c3.err || { echo C3_FAIL $c; tail -20 $O/c3.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_cus$c.json').read().strip().splitlines()[-1])
print('c3 chain_cus $c', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['launch_ms'],3), d['pivot_log_vs_oracle']['bit_identical'])"
done
DLP_CHAIN_CUS=16 DLP_LEAN_LCH=0 timeout -k 10 200 python -u tools/chain_stamps.py > $O/stamps_cus16.json 2>&1 || { echo STAMP_FAIL; tail -20 $O/stamps_cus16.json; exit 1; }
python3 -c "
import json
d=json.load(open('$O/stamps_cus16.json')); print(round(d['bench_value']), {k: round(v,1) for k,v in d['median_us'].items()})"
for w in c3r4 c3r2; do for la in 0 1; do
timeout -k 10 300 python -u bench.py --workload $w --lookahead $la --no-cpu-baseline --no-eager-window --no-pivot-window > $O/${w}_la$la.json 2> $O/$w.err || { echo FAIL $w $la; tail -20 $O/$w.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/${w}_la$la.json').read().strip().splitlines()[-1]); b=d['block']
print('$w la$la', round(d['value']), d['exchange'], 'form', d['geometry']['form'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'chain', b['chain_us_per_pivot'])"
done; done
for c in 0 16; do
DLP_CHAIN_CUS=$c timeout -k 10 300 python -u bench.py --form 23 --no-cpu-baseline --no-eager-window --no-pivot-window > $O/c3_f23_cus$c.json 2> $O/c3.err || { echo C3F23_FAIL $c; tail -20 $O/c3.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_f23_cus$c.json').read().strip().splitlines()[-1])
print('c3 form23 chain_cus $c', round(d['value']), round(d['ms_per_step'],3), round(d['roofline']['launch_ms'],3), d['pivot_log_vs_oracle']['bit_identical'])"
done
for la in 0 1 0 1; do
timeout -k 10 300 python -u bench.py --workload c3r8 --lookahead $la --no-cpu-baseline --no-eager-window --no-pivot-window > $O/c3r8_la$la.json 2> $O/c3r8.err || { echo FAIL c3r8 $la; tail -20 $O/c3r8.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3r8_la$la.json').read().strip().splitlines()[-1]); b=d['block']
print('c3r8 la$la', round(d['value']), d['exchange'], 'form', d['geometry']['form'], 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'chain', b['chain_us_per_pivot'])"
done
DLP_LEAN_LCH=0 timeout -k 10 200 python -u tools/chain_stamps.py --workload c3r8 --lookahead 1 > $O/stamps_c3r8.json 2>&1 || { echo STAMP_FAIL; tail -20 $O/stamps_c3r8.json; exit 1; }
python3 -c "
import json
d=json.load(open('$O/stamps_c3r8.json')); print('stamps c3r8', round(d['bench_value']), {k: round(v,1) for k,v in d['median_us'].items()})"
DLP_TRACE_CREATE=1 timeout -k 10 120 python -u tools/c1_overhead.py > $O/c1_overhead.json 2> $O/c1_stages.txt || { echo C1_FAIL; tail $O/c1_stages.txt; exit 1; }
tail -9 $O/c1_stages.txt
