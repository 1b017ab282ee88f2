#!/bin/bash
# GPU box: parity tests + bench for each aggregate tile geometry.
set -o pipefail
mkdir -p gpurun_out
for g in S M L; do
  PSG_GEOMETRY=$g timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$g.log 2>&1
  rc=$?; echo "geo $g pytest rc=$rc: $(tail -1 gpurun_out/pytest_$g.log)"
  [ $rc -ne 0 ] && exit $rc
  PSG_GEOMETRY=$g timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$g.json 2> gpurun_out/bench_$g.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench $g rc=$rc"; tail -5 gpurun_out/bench_$g.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$g.json'));r=d['roofline'];print('geo $g', '%.3e kv/s'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'agg %.3f ms'%r['kernel_ms'], 'part %.3f ms'%r['partition_ms'], 'achieved %.0f GB/s'%r['achieved'], 'copy %.0f'%r['measured_copy_GBps'])"
done
