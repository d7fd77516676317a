#!/bin/bash
# r04u: the tuning knobs against the default path (child processes)
set -o pipefail
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_knobs.py -m gpu > $O/knobs.log 2>&1 || { echo KNOB_FAIL; grep -E "FAIL|Error|assert" $O/knobs.log | head -30; tail -40 $O/knobs.log; exit 1; }
tail -12 $O/knobs.log
