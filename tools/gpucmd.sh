# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
R=r04; O=gpurun_out/$R; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_nway_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/nway_test.log 2>&1 || { echo TESTFAIL; tail -30 $O/nway_test.log; exit 1; }
tail -1 $O/nway_test.log
PSG_LIB_PATH=build/nwrank/libpsg.so timeout -k 10 300 python3 -u -m pytest tests/test_nway_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/nway_test_rank.log 2>&1 || { echo TESTFAIL rank; tail -30 $O/nway_test_rank.log; exit 1; }
tail -1 $O/nway_test_rank.log
for v in default rank default rank; do
  L=""; [ $v = rank ] && L=build/nwrank/libpsg.so
  PSG_LIB_PATH=$L timeout -k 10 300 python3 tools/nway_probe.py > $O/nway_probe.log 2>&1 || { echo "probe failed"; tail -5 $O/nway_probe.log; exit 1; }
  echo "$v $(grep batch $O/nway_probe.log)"
done
PSG_LIB_PATH=build/nwrankprof/libpsg.so timeout -k 10 300 python3 tools/nway_probe.py --prof --reps 3 > $O/nway_prof_rank.log 2>&1 || { echo "prof failed"; tail -5 $O/nway_prof_rank.log; exit 1; }
tail -9 $O/nway_prof_rank.log
echo done
