#!/bin/bash
# GPU box: parity once, then bench each streaming-kernel variant.
# Any failing GPU step ends the script (no further GPU work after a fault).
set -o pipefail
PSG_KERNEL=${K:-7} timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_sweep.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/pytest_sweep.log)"
[ $rc -eq 0 ] || exit $rc
for v in ${1:-0 1 2 3 4 5}; do
  PSG_KERNEL=${K:-7} PSG_STREAM2_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/pytest_v$v.log 2>&1 || { echo "variant $v parity failed"; tail -15 gpurun_out/pytest_v$v.log; exit 1; }
  PSG_KERNEL=${K:-7} PSG_STREAM_VARIANT=$v PSG_STREAM2_VARIANT=$v timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/sv_$v.json 2> gpurun_out/sv_$v.err || { echo "variant $v failed"; tail -3 gpurun_out/sv_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/sv_$v.json'));r=d['roofline'];print('variant $v: %.3e kv/s agg %.3f ms part %.3f ms  %.0f GB/s'%(d['value'],r['kernel_ms'],r['partition_ms'],r['achieved']))"
done
