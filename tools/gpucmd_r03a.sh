mkdir -p gpurun_out/r03a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/r03a/gputest.log 2>&1
rc=$?; tail -3 gpurun_out/r03a/gputest.log; grep -E "^FAILED|Error" gpurun_out/r03a/gputest.log | head -5
[ $rc -eq 0 ] || exit $rc
NOTEST=1 WLS="cfg2 cfg3 cfg5" tools/quick_bench.sh gpurun_out/r03a || exit 1
PSG_LIB_PATH=$PWD/build/phases/libpsg.so timeout -k 10 300 python3 tools/phases.py > gpurun_out/r03a/phases_cfg2.json || exit 1
PSG_LIB_PATH=$PWD/build/phases/libpsg.so timeout -k 10 300 python3 tools/phases.py --workload cfg3 > gpurun_out/r03a/phases_cfg3.json
