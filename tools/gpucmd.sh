# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_nway_gpu.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "nway or union" > $O/test_nw.log 2>&1 || { echo TESTFAIL; tail -30 $O/test_nw.log; exit 1; }
echo "tests $(tail -1 $O/test_nw.log)"
for rep in 1 2; do
timeout -k 10 300 python3 tools/nway_probe.py > $O/nw.txt 2>&1 || { echo FAIL; tail -5 $O/nw.txt; exit 1; }
echo "$rep $(grep batch $O/nw.txt | tail -1)"
done
timeout -k 10 300 python3 tools/run_rows.py > $O/rows.json 2> $O/rows.err || { echo ROWSFAIL; tail -5 $O/rows.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rows.json'));r=d.get('rows',d);[print(k,'%.4f ms'%r[k]['ms'],'frac %.3f'%r[k]['frac']) for k in ('key_union','nway_merge_1agg')]"

timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "cfg5_shard or partition or random or cfg2_full" > $O/test_pt.log 2>&1 || { echo TESTFAIL2; tail -30 $O/test_pt.log; exit 1; }
echo "tests2 $(tail -1 $O/test_pt.log)"
bash tools/ab_run.sh "intree" "cfg2 cfg5" || exit 1
echo done
