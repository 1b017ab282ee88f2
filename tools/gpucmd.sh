# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_nway_gpu.py tests/test_wire.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "nway or union or snappy or compress or wire or cache" > $O/test_nw.log 2>&1 || { echo TESTFAIL; tail -30 $O/test_nw.log; exit 1; }
echo "tests $(tail -1 $O/test_nw.log)"
timeout -k 10 300 python3 tools/run_rows.py > $O/rows.json 2> $O/rows.err || { echo ROWSFAIL; tail -5 $O/rows.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rows.json'));r=d.get('rows',d);[print(k,'%.4f ms'%r[k]['ms'],'frac %.3f'%r[k]['frac']) for k in r]"
timeout -k 10 300 python3 tools/e2e/run_e2e.py 7 compressed,pinned > $O/e2e.json 2> $O/e2e.err || { echo E2EFAIL; tail -5 $O/e2e.err; exit 1; }
cat $O/e2e.json | head -c 1500; echo
echo done
