#!/bin/bash
# r06x: kernel trace of the shipped C3 default (grouped-ring selection, 4-row pass groups) and of c3r8
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06x; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in c3 c3r8; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$w -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --workload $w > $O/trace_bench_$w.json 2> $O/trace_$w.err || { tail -20 $O/trace_$w.err; exit 1; }
done
cd $R
for w in c3 c3r8; do
  k=$(find $O/trace_$w -name "*kernel_trace.csv" | head -1); st=$(find $O/trace_$w -name "*kernel_stats.csv" | head -1)
  python3 tools/kernel_timeline.py $k 3 > $O/timeline_$w.json && cp $st $O/${w}_kernel_stats.csv
  python3 - $O/timeline_$w.json <<'PY'
import json,sys
for b in json.load(open(sys.argv[1])):
    m=lambda v: round(sum(v)/max(len(v),1),1)
    print(sys.argv[1].split('/')[-1], 'block', b['block_us'], 'pass', b['pass_us'], 'during', b['pivots_during_pass'], 'ratio', m(b['ratio_us']), 'prow', m(b['prow_us']), 'period', m(b['period_us']), 'chain_busy', b['chain_busy_us'], 'end_after_pass', b['chain_end_after_pass_us'])
PY
done
echo done
