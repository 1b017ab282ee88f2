# deferred-literal snappy: wire tests, e2e compressed mode, snappy rows
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_wire.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python3 tools/e2e/run_e2e.py 5 > $O/e2e.json 2> $O/e2e.err || { echo "e2e failed"; tail -5 $O/e2e.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/e2e.json'));[print(k,'%.3g'%v['value'],'%.3f ms'%v['ms_per_aggregate'],v.get('frac_of_link')) for k,v in d['modes'].items()]"
timeout -k 10 300 python3 tools/run_rows.py > $O/rows.json 2> $O/rows.err || { echo "rows failed"; tail -5 $O/rows.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rows.json'));[print(k,'%.4f ms'%v['ms'],'%.1f GB/s'%v['GBps']) for k,v in d.items()]"
