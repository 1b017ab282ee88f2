# r03 step b: new GPU tests, the phase split, and the full default bench line
mkdir -p gpurun_out/r03b
timeout -k 10 300 python -u -m pytest tests/test_nway_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r03b/nway.log 2>&1
rc=$?; tail -3 gpurun_out/r03b/nway.log; grep -E "^FAILED|Error" gpurun_out/r03b/nway.log | head -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 180 --timeout-method thread -k "dense_slice or nan_payload or seams or extreme or round_forms or partition_modes or packed_rounds" > gpurun_out/r03b/newtests.log 2>&1
rc=$?; tail -3 gpurun_out/r03b/newtests.log; grep -E "^FAILED|Error" gpurun_out/r03b/newtests.log | head -5
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
PSG_LIB_PATH=$PWD/build/phases/libpsg.so timeout -k 10 300 python3 tools/phases.py > gpurun_out/r03b/phases_cfg2.json || exit 1
PSG_LIB_PATH=$PWD/build/phases/libpsg.so timeout -k 10 300 python3 tools/phases.py --workload cfg3 > gpurun_out/r03b/phases_cfg3.json || exit 1
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/r03b/bench.json 2> gpurun_out/r03b/bench.err || { tail -5 gpurun_out/r03b/bench.err; exit 1; }
cat gpurun_out/r03b/phases_cfg2.json
