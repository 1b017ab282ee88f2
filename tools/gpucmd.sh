# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
R=r04; O=gpurun_out/$R; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_nway_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/nway_test.log 2>&1 || { echo TESTFAIL; tail -30 $O/nway_test.log; exit 1; }
tail -1 $O/nway_test.log
timeout -k 10 300 python3 tools/nway_probe.py > $O/nway_probe.log 2>&1 || { echo "probe failed"; tail -5 $O/nway_probe.log; exit 1; }
tail -1 $O/nway_probe.log
PSG_LIB_PATH=build/nwprof/libpsg.so timeout -k 10 300 python3 tools/nway_probe.py --prof --reps 3 > $O/nway_prof.log 2>&1 || { echo "probe failed"; tail -5 $O/nway_prof.log; exit 1; }
tail -9 $O/nway_prof.log
echo done
