#!/bin/bash
# GPU box: ablation of the v4 aggregate kernel phases (geometry M)
set -o pipefail
for mode in 1 2 3 0; do
  PSG_KERNEL=4 PSG_AGG_MODE=$mode PSG_GEOMETRY=${GEO:-M} timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/abl_$mode.json 2> gpurun_out/abl_$mode.err || { echo "mode $mode failed"; tail -3 gpurun_out/abl_$mode.err; }
  python -c "import json;d=json.load(open('gpurun_out/abl_$mode.json'));r=d['roofline'];print('mode $mode agg %.3f ms achieved %.0f GB/s'%(r['kernel_ms'],r['achieved']))" 2>/dev/null
done
