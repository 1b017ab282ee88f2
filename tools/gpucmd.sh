# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05l; mkdir -p $O
PSG_LIB_PATH=$PWD/build/fr2/libpsg.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_fr2.log 2>&1 || { echo FR2 TESTS FAILED; tail -30 $O/tests_fr2.log; exit 1; }
echo "fr2 $(tail -1 $O/tests_fr2.log)"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
tools/ab_run.sh "fr0 fr1 fr2" "cfg2 cfg5" > $O/ab.txt 2>&1 || { echo AB FAILED; cat $O/ab.txt; exit 1; }
cat $O/ab.txt
