#!/bin/bash
# GPU box: parity + bench for kernel/geometry combinations: tools/kern_sweep.sh "3:M 3:L 2:L"
set -o pipefail
mkdir -p gpurun_out
for kg in ${1:-"3:S 3:M 3:L"}; do
  k=${kg%%:*}; g=${kg##*:}
  PSG_KERNEL=$k PSG_GEOMETRY=$g timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_$k$g.log 2>&1
  rc=$?; echo "k$k geo $g pytest rc=$rc: $(tail -1 gpurun_out/pytest_$k$g.log)"
  [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_$k$g.log | head -20; exit $rc; }
  PSG_KERNEL=$k PSG_GEOMETRY=$g timeout -k 10 300 python bench.py --no-cpu-baseline $2 > gpurun_out/bench_$k$g.json 2> gpurun_out/bench_$k$g.err
  rc=$?; [ $rc -ne 0 ] && { echo "bench $k$g rc=$rc"; tail -5 gpurun_out/bench_$k$g.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$k$g.json'));r=d['roofline'];print('k$k geo $g', '%.3e kv/s'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'agg %.3f ms'%r['kernel_ms'], 'part %.3f ms'%r['partition_ms'], 'achieved %.0f GB/s'%r['achieved'], 'copy %.0f'%r['measured_copy_GBps'])"
done
