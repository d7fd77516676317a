#!/bin/bash
# r05a (second part): the cache-release test, the default bench on this round's box, the C5 bench line
set -o pipefail
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_release_cached_memory" -x -v --timeout 120 --timeout-method thread > $O/release.log 2>&1 || { echo FAIL release; tail -40 $O/release.log; exit 1; }
tail -3 $O/release.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo FAIL bench; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('c3', round(d['value']), 'pass', d['roofline']['launch_ms'], d['roofline']['frac'])"
timeout -k 10 200 python -u bench.py --workload c5 --cpu-seconds 5 > $O/c5.json 2> $O/c5.err || { echo FAIL c5; tail -20 $O/c5.err; exit 1; }
tail -c 1500 $O/c5.json
bash tools/runs/r05b.sh
