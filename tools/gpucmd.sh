# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
R=$GRAFT_REPO_ROOT
PSG_LIB_PATH=$R/build/c1/libpsg.so timeout -k 10 300 python3 -u -m pytest tests/test_freq_filter.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_c1.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests_c1.log; exit 1; }
echo "c1 $(tail -1 $O/tests_c1.log)"
for rep in 1 2; do for v in c0 c1; do
  PSG_LIB_PATH=$R/build/$v/libpsg.so timeout -k 10 300 python3 tools/run_rows.py countmin > $O/rows_$v.json 2> $O/rows_$v.err || { echo FAIL $v; tail -5 $O/rows_$v.err; exit 1; }
  echo "$rep $v $(python3 -c "import json;d=json.load(open('$O/rows_$v.json'));print(d['countmin_insert']['ms'], d['countmin_query']['ms'])")"
done; done
cd /tmp && PSG_LIB_PATH=$R/build/c1/libpsg.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_c1 -o run -- python3 $R/tools/run_rows.py countmin > $R/$O/kt_c1.log 2>&1 || { echo KT FAIL; exit 1; }
cd $R; grep -i "cm_" $O/kt_c1/run_kernel_stats.csv | cut -d, -f1-4
echo done
