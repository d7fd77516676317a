#!/bin/bash
# r04p: kernel trace of c3r8 and C3 under lookahead (per-launch start/end, no stamps), C1 teardown
set -o pipefail
O=gpurun_out/r04p; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in c3r8 c3; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/kt_$w -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload $w --steps 4 --warmup 2 --no-cpu-baseline --no-eager-window --no-pivot-window > $GRAFT_REPO_ROOT/$O/kt_$w.json 2> $GRAFT_REPO_ROOT/$O/kt_$w.err || { echo KT_FAIL $w; tail -20 $GRAFT_REPO_ROOT/$O/kt_$w.err; exit 1; }
tail -1 $GRAFT_REPO_ROOT/$O/kt_$w.json | cut -c1-200
done
cd $GRAFT_REPO_ROOT
DLP_TRACE_CREATE=1 timeout -k 10 120 python -u tools/c1_overhead.py > $O/c1_overhead.json 2> $O/c1_stages.txt || { echo C1_FAIL; tail $O/c1_stages.txt; exit 1; }
tail -16 $O/c1_stages.txt
ls -R $O | head -30
