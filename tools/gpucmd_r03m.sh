# half-run fold (padded round tables): parity, then A/B vs HEAD
set -o pipefail
O=gpurun_out/r03m; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 600 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for rep in 1 2; do
for lib in "" build/base/libpsg.so; do
  for w in cfg2 cfg3; do
    wa="--workload $w"; [ $w = cfg2 ] && wa="--no-cfg5"
    PSG_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-check $wa --steps 10 > $O/ab.json 2> $O/ab.err || { echo FAIL; tail -3 $O/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab.json'));r=d['roofline'];print('[$lib] $w kern %.4f part %.4f frac %.3f step %.4f'%(r['kernel_ms'],r['partition_ms'],r['frac'],d['ms_per_step']))"
  done
done
done
