#!/bin/bash
# Engine clock and power while the C3 bench runs (run through gpurun from the repo root):
#   tools/clock_probe.sh <tag> [bench args...]
# rocm-smi samples every ~0.5 s beside a bench.py run, and one rocprofv3 --pmc pass of
# GRBM_COUNT / GRBM_GUI_ACTIVE + SQ_CYCLES / SQ_BUSY_CYCLES for the pass kernel.
set -o pipefail
R=$(pwd); TAG=$1; shift
OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-eager-window --steps 60 "$@" > $OUT/clk_bench.json 2> $OUT/clk_bench.err &
B=$!
for i in $(seq 1 24); do
  sleep 0.5
  kill -0 $B 2>/dev/null || break
  (echo "t=$i"; timeout 10 rocm-smi --showclocks --showpower --showuse 2>&1 | grep -Ei "sclk|fclk|mclk|power|GPU use") >> $OUT/clk_smi.txt
done
wait $B || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE SQ_CYCLES SQ_BUSY_CYCLES --output-format csv \
    -d $OUT/grbm -o run -- python3 $R/bench.py --no-cpu-baseline --no-pivot-window --no-eager-window \
    --steps 6 --warmup 2 "$@" > $OUT/grbm_bench.json 2> $OUT/grbm.err || exit 1
cd $R && python3 tools/sq_summary.py $OUT/grbm pass_d_kernel > $OUT/grbm_summary.json; cat $OUT/grbm_summary.json
