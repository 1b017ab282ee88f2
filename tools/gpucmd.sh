# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 120 ./tools/calib/stride_read > $O/stride.txt 2>&1 || { echo STRIDE FAILED; cat $O/stride.txt; exit 1; }
cat $O/stride.txt
timeout -k 10 300 python3 -u -m pytest tests/test_freq_filter.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
timeout -k 10 300 python3 tools/run_rows.py countmin > $O/rows.json 2> $O/rows.err || { echo ROWS FAILED; tail $O/rows.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rows.json'));[print(k,'%.4f ms'%v['ms']) for k,v in d.items()]"
ROWS=countmin PASSES="1 2" tools/pmc_rows.sh $O/pmc > $O/pmc.log 2>&1 || { echo PMC FAILED; cat $O/pmc.log; exit 1; }
python3 - <<'PY'
import json
d=json.load(open('gpurun_out/r06k/pmc/summary.json'))
for k,v in d.items():
    if 'cm_' in k: print(k, {c: v.get(c) for c in ('FETCH_SIZE','WRITE_SIZE')})
PY
