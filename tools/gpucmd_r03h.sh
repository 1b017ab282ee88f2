# sorted fold: parity, then A/B timing (0 = round fold, 0x200000 = sorted fold)
mkdir -p gpurun_out/r03h
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -v --timeout 180 --timeout-method thread -k "sorted_fold or round_forms or extreme" > gpurun_out/r03h/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r03h/tests.log; grep -E "^FAILED" gpurun_out/r03h/tests.log | head -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for f in 0 0x200000 0 0x200000; do
  for w in cfg2 cfg3; do
    a="--workload $w"; [ $w = cfg2 ] && a="--no-cfg5"
    ff=$f; [ $w = cfg3 ] && [ $f != 0 ] && ff=$((f | 0x10000))
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-check $a --steps 10 --plan-flags $ff > gpurun_out/r03h/ab.json 2> gpurun_out/r03h/ab.err || { echo FAIL; tail -3 gpurun_out/r03h/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r03h/ab.json'));r=d['roofline'];print('$ff $w kern %.4f part %.4f frac %.3f'%(r['kernel_ms'],r['partition_ms'],r['frac']))"
  done
done
PSG_LIB_PATH=$PWD/build/phases/libpsg.so timeout -k 10 300 python3 tools/phases.py > gpurun_out/r03h/phases_cfg2.json || exit 1
cat gpurun_out/r03h/phases_cfg2.json
