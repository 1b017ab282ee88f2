# snappy parse clock split (diagnostic build)
set -o pipefail
O=gpurun_out/r03q; mkdir -p $O
PSG_LIB_PATH=$PWD/build/sprof/libpsg.so timeout -k 10 300 python3 tools/snappy_prof.py > $O/sprof.json 2> $O/sprof.err || { echo FAIL; tail -5 $O/sprof.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/sprof.json'))
for k,v in d.items():
  print(k, '%.4f ms'%v['ms'])
  for p in v['per_part'][:4]: print(p)
"
timeout -k 10 600 python3 -u -m pytest tests/test_wire.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 tools/e2e/run_e2e.py 5 compressed,pinned,pinned_hold > $O/e2e.json 2> $O/e2e.err || { echo "e2e failed"; tail -5 $O/e2e.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/e2e.json'));[print(k,'%.3g'%v['value'],'%.3f ms'%v['ms_per_aggregate']) for k,v in d['modes'].items()]"
