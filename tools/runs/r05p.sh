#!/bin/bash
# r05p: chain phase stamps at C3 (DLP_CHAIN_STAMPS; diagnostics, never a timed figure) with the form-21 pass and
# with form 22; then the default bench once more on this box
set -o pipefail
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 300 python -u tools/chain_stamps.py > $O/stamps_f21.json 2> $O/stamps_f21.err || { tail -20 $O/stamps_f21.err; exit 1; }
cat $O/stamps_f21.json
timeout -k 10 300 python -u tools/chain_stamps.py --form 22 > $O/stamps_f22.json 2> $O/stamps_f22.err || { tail -20 $O/stamps_f22.err; exit 1; }
cat $O/stamps_f22.json
