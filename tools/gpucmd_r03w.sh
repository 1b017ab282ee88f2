# packed kernel: one 256-push group per tile (g256) vs 128-push groups (g128, HEAD)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03w; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_exchange_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
bash tools/ab_run.sh "g128 g256" "cfg5" 2>&1 | tee $O/ab.txt
bash tools/pmc_rows.sh gpurun_out/r03w/pmc_rows > gpurun_out/r03w/pmc_rows.log 2>&1 || { echo "pmc rows failed"; tail -5 gpurun_out/r03w/pmc_rows.log; exit 1; }
