# gather restructure (requests first, register repeat test); GPU tests; rows
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03y; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python3 tools/run_rows.py > $O/rows.json 2> $O/rows.err || { echo "rows failed"; tail -5 $O/rows.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rows.json'));[print(k,'%.4f ms'%v['ms'],'frac %.3f'%v['frac']) for k,v in d.items()]"
