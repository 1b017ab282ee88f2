mkdir -p gpurun_out/r03e
for i in 1 2; do
timeout -k 10 600 python3 -X faulthandler bench.py --no-cpu-baseline > gpurun_out/r03e/bench$i.json 2> gpurun_out/r03e/bench$i.err
echo "bench$i rc=$? bytes=$(wc -c < gpurun_out/r03e/bench$i.json)"; tail -3 gpurun_out/r03e/bench$i.err
done
