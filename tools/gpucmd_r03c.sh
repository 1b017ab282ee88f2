# r03 step c: nway + context union + whole-cfg5 tests, phase split, bench line
mkdir -p gpurun_out/r03c
timeout -k 10 300 python -u -m pytest tests/test_nway_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/r03c/nway.log 2>&1
rc=$?; tail -3 gpurun_out/r03c/nway.log; grep -E "^FAILED|Error" gpurun_out/r03c/nway.log | head -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v --timeout 600 --timeout-method thread -k "cfg5_whole" > gpurun_out/r03c/cfg5whole.log 2>&1
rc=$?; tail -3 gpurun_out/r03c/cfg5whole.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PSG_LIB_PATH=$PWD/build/phases/libpsg.so timeout -k 10 300 python3 tools/phases.py > gpurun_out/r03c/phases_cfg2.json || exit 1
PSG_LIB_PATH=$PWD/build/phases/libpsg.so timeout -k 10 300 python3 tools/phases.py --workload cfg3 > gpurun_out/r03c/phases_cfg3.json || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cfg5 --plan-flags 0x20000 > gpurun_out/r03c/cfg2_g64.json 2> gpurun_out/r03c/cfg2_g64.err || exit 1
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/r03c/bench.json 2> gpurun_out/r03c/bench.err || { tail -5 gpurun_out/r03c/bench.err; exit 1; }
cat gpurun_out/r03c/phases_cfg2.json
