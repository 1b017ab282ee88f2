# GPU tests (growing value-array list, static-keys plans); 1-bucket-per-slot A/B (cfg2)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
bash tools/ab_run.sh "nb2 nb1" "cfg2" 2>&1 | tee $O/ab.txt
bash tools/gpucmd_r03t.sh
