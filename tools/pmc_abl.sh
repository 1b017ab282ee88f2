#!/bin/bash
# GPU box: SQ/LDS counters of v7 variant 10 and its ablations (21: no fold,
# 22: no search).  Each run under its own limit; first failure ends it.
set -o pipefail
for v in ${1:-10 21 22}; do
  SV=$v PASSES="${PASSES:-4 5 6 7 9}" ./tools/pmc2.sh "7:S" > gpurun_out/pmc_abl_$v.log 2>&1 || { echo "pmc variant $v failed"; tail -5 gpurun_out/pmc_abl_$v.log; exit 1; }
  rm -rf gpurun_out/pmc_abl_$v && mv gpurun_out/pmc2/k7S gpurun_out/pmc_abl_$v
  python3 -c "
import json; d=json.load(open('gpurun_out/pmc_abl_$v/summary.json'))['counters']['stream2_kernel']
print('v$v', ' '.join('%s=%.3g'%(k,d[k]) for k in sorted(d)))"
done
