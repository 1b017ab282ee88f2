#!/bin/bash
# GPU box: parity once, then bench each streaming-kernel variant
set -o pipefail
PSG_KERNEL=${K:-6} timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_6.log 2>&1; echo "pytest rc=$?: $(tail -1 gpurun_out/pytest_6.log)"
for v in ${1:-0 1 2 3 4 5}; do
  PSG_KERNEL=${K:-6} PSG_STREAM_VARIANT=$v PSG_STREAM2_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/sv_$v.json 2> gpurun_out/sv_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/sv_$v.err; continue; }
  python -c "import json;d=json.load(open('gpurun_out/sv_$v.json'));r=d['roofline'];print('variant $v: %.3e kv/s agg %.3f ms part %.3f ms  %.0f GB/s'%(d['value'],r['kernel_ms'],r['partition_ms'],r['achieved']))"
done
