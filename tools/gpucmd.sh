# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
R=r04; OUT=gpurun_out/$R; mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_freq_filter.py -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/freq_test.log 2>&1 || { echo TESTFAIL; tail -30 $OUT/freq_test.log; exit 1; }
tail -1 $OUT/freq_test.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace_rows3 -o run -- python3 tools/run_rows.py > $OUT/rows3.json 2> $OUT/rows3.err || { echo "rows failed"; tail -5 $OUT/rows3.err; exit 1; }
python3 -c "
import json;d=json.load(open('$OUT/rows3.json'))
print({k:(round(v['ms'],4),round(v['frac'],3)) for k,v in d.items() if k.startswith('countmin')})"
grep -i "cm_bin" $OUT/ktrace_rows3/run_kernel_stats.csv | cut -d, -f1-4
PASSES="1 2" ./tools/pmc_rows.sh $OUT/pmc_rows3 > $OUT/pmc_rows3.log 2>&1 || { echo "pmc rows failed"; tail -5 $OUT/pmc_rows3.log; exit 1; }
python3 -c "
import json;r=json.load(open('$OUT/pmc_rows3/summary.json'))['counters']
print({k:round(v.get('hbm_bytes_corrected',0)/1e9,3) for k,v in r.items() if k.startswith('cm_')})"
echo done
