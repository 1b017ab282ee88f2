#!/bin/bash
# GPU box: SQ counters of the v10 rows kernel (passes 4-9 of tools/pmc2.sh).
set -o pipefail
PASSES="${PASSES:-4 5 6 7 8 9}" ./tools/pmc2.sh "10:S" > gpurun_out/pmc_rows.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_rows.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/pmc2/k10S/summary.json'))['counters']
for k,v in d.items(): print(k, ' '.join('%s=%.4g'%(c,v[c]) for c in sorted(v)))"
