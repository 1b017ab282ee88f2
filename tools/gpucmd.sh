# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/test_all.log 2>&1 || { echo TESTFAIL; tail -30 $O/test_all.log; exit 1; }
echo "tests $(tail -1 $O/test_all.log)"
for r in 1 2; do
timeout -k 10 300 python3 tools/e2e/run_e2e.py 7 pageable,pinned,pinned_hold,compressed > $O/e2e.json 2> $O/e2e.err || { echo E2EFAIL; tail -5 $O/e2e.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/e2e.json'));print(' '.join('%s %.3f'%(k,v['ms_per_aggregate']) for k,v in d['modes'].items()))"
done
echo done
