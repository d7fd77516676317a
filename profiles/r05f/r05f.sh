#!/bin/bash
# r05f: rocprofv3 kernel trace + stats of the default bench (C3, form 21) and of --form 22, then the PMC
# FETCH_SIZE / WRITE_SIZE passes of the default (the shipped kernel's traffic, re-taken this round)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r05f; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_f21 -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window > $O/trace_f21_bench.json 2> $O/trace_f21.err || { tail -20 $O/trace_f21.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_f22 -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --form 22 > $O/trace_f22_bench.json 2> $O/trace_f22.err || { tail -20 $O/trace_f22.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/pmc_write.json 2> $O/pmc_write.err || { tail -20 $O/pmc_write.err; exit 1; }
find $O -name "*kernel_stats.csv" | head
echo done
