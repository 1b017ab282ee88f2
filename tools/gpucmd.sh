# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
PSG_LIB_PATH=$PWD/build/ga1/libpsg.so timeout -k 10 300 python3 -u -m pytest tests/test_nway_gpu.py tests/test_gpu_parity.py -k "nway or union or NWay" -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_ga1.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests_ga1.log; exit 1; }
echo "ga1 $(tail -1 $O/tests_ga1.log)"
for rep in 1 2; do for v in ga0 ga1; do
  PSG_LIB_PATH=$PWD/build/$v/libpsg.so timeout -k 10 300 python3 tools/nway_probe.py > $O/nw_$v.txt 2> $O/nw_$v.err || { echo FAIL $v; tail -5 $O/nw_$v.err; exit 1; }
  PSG_LIB_PATH=$PWD/build/$v/libpsg.so timeout -k 10 300 python3 tools/run_rows.py nway > $O/rows_$v.json 2> $O/rows_$v.err || { echo FAIL rows $v; tail -5 $O/rows_$v.err; exit 1; }
  echo "$rep $v $(grep batch $O/nw_$v.txt) $(python3 -c "import json;d=json.load(open('$O/rows_$v.json'));print('union %.4f 1agg %.4f'%(d['key_union']['ms'],d['nway_merge_1agg']['ms']))")"
done; done
echo done
