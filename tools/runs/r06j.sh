#!/bin/bash
# r06j: kernel traces of the condensed rank geometries c3r8 / c3r4 (per-pivot chain timeline)
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r06j; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in c3r8 c3r4; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$w -o run -- \
    python3 $R/bench.py --workload $w --no-cpu-baseline --no-eager-window --no-pivot-window > $O/${w}_bench.json 2> $O/${w}.err || { tail -20 $O/${w}.err; exit 1; }
K=$(find $O/$w -name "*kernel_trace.csv" | head -1)
python3 $R/tools/kernel_timeline.py $K 3 > $O/${w}_timeline.json
cp $(find $O/$w -name "*kernel_stats.csv" | head -1) $O/${w}_kernel_stats.csv
rm -rf $O/$w
done

timeout -k 10 600 python -u -m pytest tests/test_gpu_knobs.py -v --timeout 300 --timeout-method thread > $O/knobs.log 2>&1 || { grep -E "FAILED|^E " $O/knobs.log | head; exit 1; }
tail -1 $O/knobs.log
