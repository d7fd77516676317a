#!/bin/bash
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r03j; mkdir -p $OUT
bash tools/gpu_profile.sh r03j_prof || exit 1
python3 tools/pmc_summary.py gpurun_out/r03j_prof pass_d_kernel $OUT/c3_pass_pmc_traffic.json "form 21, 768-row bands, ld 65664, nt, lookahead, band publication (sc1 stores)" || exit 1
timeout -k 10 300 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
cat $OUT/bench_default.json
