# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_wire.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "snappy or compress or wire or cache or pinned or hold" > $O/test_c.log 2>&1 || { echo TESTFAIL; tail -30 $O/test_c.log; exit 1; }
echo "tests $(tail -1 $O/test_c.log)"
timeout -k 10 300 python3 tools/e2e/run_e2e.py 7 compressed,pinned > $O/e2e.json 2> $O/e2e.err || { echo E2EFAIL; tail -5 $O/e2e.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/e2e.json'));[print(k,v['ms_per_aggregate']) for k,v in d['modes'].items()]"
timeout -k 10 300 python3 tools/e2e/run_e2e.py 7 compressed,pinned > $O/e2e.json 2> $O/e2e.err || { echo E2EFAIL; tail -5 $O/e2e.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/e2e.json'));[print(k,v['ms_per_aggregate']) for k,v in d['modes'].items()]"
echo done
