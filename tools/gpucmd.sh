# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "seams or growing or random or cfg2_full or cfg5_shard or packed or dense or cfg4" > $O/test_up.log 2>&1 || { echo TESTFAIL; tail -30 $O/test_up.log; exit 1; }
echo "tests $(tail -1 $O/test_up.log)"
bash tools/ab_run.sh "base up" "cfg2 cfg5 cfg3" || exit 1
echo done
