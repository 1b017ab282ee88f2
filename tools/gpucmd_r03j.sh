# tile rows: parity of the tile kernel paths, then A/B rows vs PSG_NO_ROWS on cfg2 / cfg3
mkdir -p gpurun_out/r03j
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "not whole_workload" > gpurun_out/r03j/tests.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/r03j/tests.log; exit 1; }
tail -3 gpurun_out/r03j/tests.log
for a in "" "--plan-flags 0x200000" "" "--plan-flags 0x200000"; do
  for w in cfg2 cfg3; do
    wa="--workload $w"; [ $w = cfg2 ] && wa="--no-cfg5"
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-check $wa --steps 10 $a > gpurun_out/r03j/ab.json 2> gpurun_out/r03j/ab.err || { echo FAIL; tail -3 gpurun_out/r03j/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r03j/ab.json'));r=d['roofline'];print('[$a] $w kern %.4f part %.4f frac %.3f step %.4f'%(r['kernel_ms'],r['partition_ms'],r['frac'],d['ms_per_step']))"
  done
done
