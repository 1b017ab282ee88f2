#!/bin/bash
set -o pipefail
for v in 10 21 22 10; do
  PSG_STREAM2_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/sv_$v.json 2> gpurun_out/sv_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/sv_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sv_$v.json'));r=d['roofline'];print('variant $v: agg %.3f ms'%(r['kernel_ms']))"
done
