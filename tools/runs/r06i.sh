#!/bin/bash
# r06i: the condensed C3 default bench's kernel trace and the PMC passes of its tableau pass; the c5 line
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06i; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/trace_bench.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/pmc_fetch.json 2> $O/pmc_fetch.err || { tail -20 $O/pmc_fetch.err; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- \
    python3 $R/bench.py --no-cpu-baseline --no-eager-window --no-pivot-window > $O/pmc_write.json 2> $O/pmc_write.err || { tail -20 $O/pmc_write.err; exit 1; }
cd $R
timeout -k 10 300 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo FAIL c5; tail -20 $O/bench_c5.err; exit 1; }
echo done
