#!/bin/bash
# r04a: the C3 rank geometry at P = 8 (c3r8) on one GPU: exchange x lookahead, chain stamps, rocprof
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r04a
mkdir -p $O
B="python -u bench.py --workload c3r8 --no-cpu-baseline --no-eager-window --no-pivot-window"
summ() { python3 -c "import json,sys;d=json.load(open('$1'));b=d['block'];print('$1'.split('/')[-1], round(d['value']), 'x', d['exchange'], 'la', b['lookahead'], 'form', d['geometry']['form'], 'rb', d['geometry']['rows_per_block'], 'block_ms', round(b['ms'],3), 'pass_ms', round(b['pass_ms'],3), 'chain_us', b['chain_us_per_pivot'])"; }
for x in peer rccl; do for la in 0 1; do
  timeout -k 10 240 $B --exchange $x --lookahead $la > $O/c3r8_${x}_la$la.json 2> $O/c3r8_${x}_la$la.err || { echo FAIL $x $la; tail -20 $O/c3r8_${x}_la$la.err; exit 1; }
  summ $O/c3r8_${x}_la$la.json
done; done
DLP_LEAN_LCH=0 timeout -k 10 200 python -u tools/chain_stamps.py --workload c3r8 --exchange peer --lookahead 1 > $O/stamps_peer_la1.json 2>&1 || { echo STAMP_FAIL; tail -20 $O/stamps_peer_la1.json; exit 1; }
cat $O/stamps_peer_la1.json
cd /tmp && export TMPDIR=/tmp
for la in 0 1; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_la$la -o run -- python3 $R/bench.py --workload c3r8 --exchange peer --lookahead $la --no-cpu-baseline --no-eager-window --no-pivot-window > $O/prof_la$la.json 2> $O/prof_la$la.err || { echo PROF_FAIL; tail -20 $O/prof_la$la.err; exit 1; }
done
cd $R
for la in 0 1; do f=$(find $O/prof_la$la -name '*kernel_stats.csv' | head -1); echo "== la$la $f"; python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:12]: print(r['Name'].replace('void dlp::(anonymous namespace)::','').split('(')[0][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2),'us', r['Percentage'][:5])
"; done
echo r04a done
