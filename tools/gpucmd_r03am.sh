# stream partition: position-guessed first splitter window vs HEAD
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03am; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
bash tools/ab_run.sh "base pguess" "cfg5" 2>&1 | tee $O/ab.txt
