# resident bucket index: parity (plan tests use it, context tests do not), A/B timing
mkdir -p gpurun_out/r03g
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q --timeout 180 --timeout-method thread -k "plan or extreme or random" > gpurun_out/r03g/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03g/tests.log; grep -E "^FAILED" gpurun_out/r03g/tests.log | head -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for f in 0 0x100000 0 0x100000; do
  for w in cfg2 cfg3; do
    a="--workload $w"; [ $w = cfg2 ] && a="--no-cfg5"
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-check $a --steps 10 --plan-flags $f > gpurun_out/r03g/ab.json 2> gpurun_out/r03g/ab.err || { echo FAIL; tail -3 gpurun_out/r03g/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r03g/ab.json'));r=d['roofline'];print('$f $w kern %.4f part %.4f frac %.3f'%(r['kernel_ms'],r['partition_ms'],r['frac']))"
  done
done
