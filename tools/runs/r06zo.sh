#!/bin/bash
# r06zo: SQ counters of the condensed C3 pass (wave states, VALU issue, effective clock)
set -o pipefail
SQ_SET=state timeout -k 10 200 bash tools/sq_counters.sh r06zo pass_q_kernel || exit 1
SQ_SET=insts timeout -k 10 200 bash tools/sq_counters.sh r06zo pass_q_kernel || exit 1
echo done
