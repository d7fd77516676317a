#!/bin/bash
# r05b: C3 pass band height vs the pass's last-round tail (257 column tiles x bands over 768 pass
# slots): 768 rows (43 bands, 14.39 rounds) vs 781 (42, 14.05), 729 (45, 15.06), 683 (48, 16.06),
# alternating
set -o pipefail
O=gpurun_out/r05b; mkdir -p $O
run() {  # tag rb
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-eager-window --no-pivot-window --rows-per-block $2 > $O/c3_$1.json 2> $O/c3_$1.err || { echo FAIL $1; tail -20 $O/c3_$1.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/c3_$1.json').read().strip().splitlines()[-1]); b=d['block']
print('$1', round(d['value']), 'block', round(b['ms'],3), 'pass', round(b['pass_ms'],3), 'frac', round(d['roofline']['frac'],4), 'rb', d['geometry']['rows_per_block'])"
}
run a768 768 && run a781 781 && run a729 729 && run a683 683 && run b768 768 && run b781 781 && run b729 729 && run b683 683
