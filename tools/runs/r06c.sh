#!/bin/bash
# r06c: condensed tableau on by default: the whole GPU suite
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --maxfail 20 --timeout-method thread > $O/suite.log 2>&1; rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/suite.log | tail -30
if [ $rc -ne 0 ]; then grep -E "^E " $O/suite.log | cut -c1-300 | head -30; exit 1; fi
