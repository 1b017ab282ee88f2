mkdir -p gpurun_out/r03d
NCCL_DEBUG=WARN timeout -k 10 600 python3 -X faulthandler bench.py --no-cpu-baseline > gpurun_out/r03d/bench.json 2> gpurun_out/r03d/bench.err
echo "bench rc=$?"; tail -5 gpurun_out/r03d/bench.err; head -c 300 gpurun_out/r03d/bench.json
