# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 400 --timeout-method thread -k "whole_workload or cfg2_full or cfg3_full" > $O/test_cfg5.log 2>&1 || { echo TESTFAIL; tail -30 $O/test_cfg5.log; exit 1; }
echo "tests $(tail -1 $O/test_cfg5.log)"
bash tools/ab_run.sh "base ed0 ed1" "cfg2 cfg3" || exit 1
echo done
