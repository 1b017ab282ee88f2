# exchange pack rewrite (own pieces into the receive buffer) + packed kernel with the resident index
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03v; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
for f in 0 0x100000 0 0x100000; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg5 --steps 10 --plan-flags $f > $O/l5.json 2> $O/l5.err || { echo "cfg5 $f failed"; tail -3 $O/l5.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/l5.json'));r=d['roofline'];print('[$f] cfg5 kern %.4f part %.4f frac %.3f step %.4f'%(r['kernel_ms'],r['partition_ms'],r['frac'],d['ms_per_step']))" | tee -a $O/ab.txt
done
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -3 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(json.dumps(d['cfg5']['modes']['unsliced']))"
