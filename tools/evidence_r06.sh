# r06 evidence on the final code (one gpurun call): GPU tests, smoke, kernel
# trace of the default bench, the cfg2 aggregate/partition traffic passes, the
# cfg3/cfg4/cfg5 side lines and the default bench line.
# usage: tools/evidence_r06.sh r06e
set -o pipefail
export TMPDIR=/tmp
R=${1:-r06e}; O=gpurun_out/$R; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --no-cpu-baseline > $O/ktrace.json 2> $O/ktrace.err || { echo "ktrace failed"; tail -5 $O/ktrace.err; exit 1; }
python3 tools/ktrace_by_grid.py $(ls $O/ktrace/*kernel_trace.csv $O/ktrace/*/*kernel_trace.csv 2>/dev/null | head -1) tile_kernel partition_kernel tile_packed > $O/ktrace_by_grid.txt || { echo "by-grid failed"; exit 1; }
grep -E "tile_kernel<float, 1, 32>.*15319040|partition_kernel.*491520" $O/ktrace_by_grid.txt || true
PASSES="1 2" timeout -k 10 400 tools/pmc2.sh $O/pmc "--prewarm-ms 0" > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
for w in cfg3 cfg4 cfg5; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload $w > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail -5 $O/bench_$w.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$w.json'));r=d['roofline'];print('$w %.4e ms %.4f kern %.4f part %.4f frac %.3f step %.3f'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['partition_ms'],r['frac'],r['step_frac']))"
done
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench %.4e ms %.4f kern %.4f part %.4f frac %.3f step %.3f'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['partition_ms'],r['frac'],r['step_frac']))"
echo done
