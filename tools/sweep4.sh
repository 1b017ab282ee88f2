#!/bin/bash
# GPU box: full GPU tests on the default kernel (v9), then each v9 variant
# (parity + bench), then v7 variant 10 for comparison.
set -o pipefail
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_s4.log 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 gpurun_out/pytest_s4.log)"
[ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_s4.log; exit $rc; }
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_$name.json 2> gpurun_out/b_$name.err || { echo "$name failed"; tail -3 gpurun_out/b_$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_$name.json'));r=d['roofline'];print('$name: %.3e kv/s agg %.3f ms part %.3f ms'%(d['value'],r['kernel_ms'],r['partition_ms']))"
}
for v in ${V4:-0 1 2 3 4 5}; do
  PSG_STREAM4_VARIANT=$v timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/pytest_s4v$v.log 2>&1 || { echo "v9 variant $v parity failed"; tail -15 gpurun_out/pytest_s4v$v.log; exit 1; }
  run s4v$v PSG_STREAM4_VARIANT=$v
done
for v in ${V2:-10}; do
  run s2v$v PSG_KERNEL=7 PSG_STREAM2_VARIANT=$v
done
