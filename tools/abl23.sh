#!/bin/bash
# GPU box: v7 variant 10 and its ablations (21 no fold, 22 + no search,
# 23 + no bucket table), then SQ counters for 10 and 23.
set -o pipefail
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_$name.json 2> gpurun_out/b_$name.err || { echo "$name failed"; tail -3 gpurun_out/b_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_$name.json'));r=d['roofline'];print('$name: %.3e kv/s agg %.3f ms part %.3f ms'%(d['value'],r['kernel_ms'],r['partition_ms']))"
}
for v in 10 21 22 23; do run s2v$v PSG_KERNEL=7 PSG_STREAM2_VARIANT=$v || exit 1; done
PSG_KERNEL=7 PASSES="4 5 6 8" ./tools/pmc_abl.sh "10 23"
