# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06za; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
for rep in 1 2; do
for v in main px0; do
  L=$PWD/parameter_server_amd/libpsg.so; [ $v = main ] || L=$PWD/build/$v/libpsg.so
  for w in cfg2 cfg5; do
    PSG_LIB_PATH=$L timeout -k 10 300 python3 bench.py --workload $w --profile-steps 20 --steps 20 > /dev/null 2> $O/err_${v}_$w.log || { echo FAIL $v $w; tail -3 $O/err_${v}_$w.log; exit 1; }
    echo "$rep $v $w $(grep 'profile run' $O/err_${v}_$w.log)"
  done
done
done
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench %.4e ms %.4f kern %.4f part %.4f frac %.3f step %.3f'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['partition_ms'],r['frac'],r['step_frac']))"
