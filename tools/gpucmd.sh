# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v; mkdir -p $O
PSG_LIB_PATH=$PWD/build/sprof/libpsg.so timeout -k 10 120 python3 tools/snappy_prof.py > $O/sprof.json 2> $O/sprof.err || { echo SPROF FAILED; tail -5 $O/sprof.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/sprof.json'))
for n,v in d.items():
  print(n, 'ms', round(v['ms'],4))
  for p in v['per_part'][:2]: print('  ', p['bytes_in'], p['tab'])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/nw -o run -- python3 tools/run_rows.py nway > $O/nway.json 2> $O/nway.err || { echo NW FAILED; tail -5 $O/nway.err; exit 1; }
python3 tools/ktrace_by_grid.py $(ls $O/nw/*kernel_trace.csv $O/nw/*/*kernel_trace.csv 2>/dev/null | head -1) nw_ | tee $O/nw_by_grid.txt
for rep in 1 2; do
for v in main sk3; do
  L=$PWD/parameter_server_amd/libpsg.so; [ $v = main ] || L=$PWD/build/$v/libpsg.so
  PSG_LIB_PATH=$L timeout -k 10 300 python3 bench.py --workload cfg3 --no-check --profile-steps 20 --steps 20 > /dev/null 2> $O/err_$v.log || { echo FAIL $v; tail -3 $O/err_$v.log; exit 1; }
  echo "$rep $v cfg3 $(grep 'profile run' $O/err_$v.log)"
done
done
PSG_LIB_PATH=$PWD/build/fsplit/libpsg.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/fsplit_tests.log 2>&1 || { echo FSPLIT TESTS FAILED; tail -30 $O/fsplit_tests.log; exit 1; }
echo "fsplit tests $(tail -1 $O/fsplit_tests.log)"
for rep in 1 2; do
for v in main fsplit; do
  L=$PWD/parameter_server_amd/libpsg.so; [ $v = main ] || L=$PWD/build/$v/libpsg.so
  PSG_LIB_PATH=$L timeout -k 10 300 python3 bench.py --workload cfg3 --profile-steps 20 --steps 20 > /dev/null 2> $O/errf_$v.log || { echo FAIL $v; tail -3 $O/errf_$v.log; exit 1; }
  echo "$rep $v cfg3 $(grep 'profile run' $O/errf_$v.log)"
done
done
bash tools/evidence_r06.sh r06f
