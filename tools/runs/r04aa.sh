#!/bin/bash
# r04aa: kernel trace of c3r8 / c3r4 with the disjoint CU split
set -o pipefail
O=gpurun_out/r04aa; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in c3r8 c3r4; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_$w -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload $w --steps 4 --warmup 2 --no-cpu-baseline --no-eager-window --no-pivot-window > $GRAFT_REPO_ROOT/$O/kt_$w.json 2> $GRAFT_REPO_ROOT/$O/kt_$w.err || { echo KT_FAIL $w; tail -20 $GRAFT_REPO_ROOT/$O/kt_$w.err; exit 1; }
tail -1 $GRAFT_REPO_ROOT/$O/kt_$w.json | cut -c1-120
done
