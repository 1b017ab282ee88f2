# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_nway_gpu.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "nway or union" > $O/test_nw.log 2>&1 || { echo TESTFAIL; tail -30 $O/test_nw.log; exit 1; }
echo "tests $(tail -1 $O/test_nw.log)"
for r in 1 2; do
timeout -k 10 300 python3 tools/run_rows.py > $O/rows.json 2> $O/rows.err || { echo ROWSFAIL; tail -5 $O/rows.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rows.json'));r=d.get('rows',d);print(' '.join('%s %.4f'%(k,r[k]['ms']) for k in ('key_union','nway_merge_1agg')))"
done
echo done
