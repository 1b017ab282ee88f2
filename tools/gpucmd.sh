# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_wire.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/test_wire.log 2>&1 || { echo TESTFAIL; tail -30 $O/test_wire.log; exit 1; }
echo "tests $(tail -1 $O/test_wire.log)"
