# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05j; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
echo "tests $(tail -1 $O/tests.log)"
tools/ab_run.sh "pf0 pf1" "cfg2 cfg5 cfg3" > $O/ab.txt 2>&1 || { echo AB FAILED; cat $O/ab.txt; exit 1; }
cat $O/ab.txt
