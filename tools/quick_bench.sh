#!/bin/bash
# GPU box: GPU tests (unless NOTEST=1), then kernel timings of cfg2 / cfg3 /
# cfg4 / cfg5 side lines (no baselines).  usage: tools/quick_bench.sh <outdir>
O=${1:-gpurun_out/quick}; mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gputest.log 2>&1
  rc=$?; tail -2 $O/gputest.log; grep -E "^FAILED|Error" $O/gputest.log | head -5
  [ $rc -eq 0 ] || exit $rc
fi
for w in ${WLS:-cfg2 cfg3 cfg4 cfg5}; do
  a="--workload $w"; [ $w = cfg2 ] && a="--no-cfg5"
  timeout -k 10 300 python3 bench.py --no-cpu-baseline $a $BARGS > $O/$w.json 2> $O/$w.err || { echo "bench $w failed"; tail -3 $O/$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$w.json'));r=d['roofline'];print('$w','%.3e'%d['value'],'ms/step %.3f kern %.3f part %.3f frac %.3f step_frac %.3f copy %s'%(d['ms_per_step'],r['kernel_ms'],r['partition_ms'],r['frac'],r['step_frac'],r['measured_copy_GBps']))"
done
