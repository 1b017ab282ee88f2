#!/bin/bash
# GPU box: v10 (rows) parity + bench over tile sizes / rows in flight.
set -o pipefail
export PSG_KERNEL=10
for cfg in ${CFGS:-1024:8 512:4}; do
  C=${cfg%%:*}; R=${cfg##*:}
  PSG_ROWS_TILE=$C PSG_ROWS_R=$R timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_rows$C.log 2>&1 || { echo "rows C=$C parity failed"; tail -30 gpurun_out/pytest_rows$C.log; exit 1; }
  echo "rows C=$C parity: $(tail -1 gpurun_out/pytest_rows$C.log)"
  PSG_ROWS_TILE=$C PSG_ROWS_R=$R timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_rows$C.$R.json 2> gpurun_out/b_rows$C.$R.err || { echo "bench $cfg failed"; tail -5 gpurun_out/b_rows$C.$R.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/b_rows$C.$R.json'));r=d['roofline'];print('rows C=$C R=$R: %.3e kv/s agg %.3f ms part %.3f ms'%(d['value'],r['kernel_ms'],r['partition_ms']))"
done
