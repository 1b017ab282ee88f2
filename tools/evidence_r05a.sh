# r05 evidence, part A (one gpurun call): GPU tests, smoke, kernel traces
# (default bench, cfg5 side line, rows), cfg2 PMC passes.  usage: tools/evidence_r05a.sh r05
set -o pipefail
export TMPDIR=/tmp
R=${1:-r05}; O=gpurun_out/$R; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --no-cpu-baseline > $O/ktrace.json 2> $O/ktrace.err || { echo "ktrace failed"; tail -5 $O/ktrace.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_cfg5 -o run -- python3 bench.py --no-cpu-baseline --workload cfg5 > $O/ktrace_cfg5.json 2> $O/ktrace_cfg5.err || { echo "ktrace cfg5 failed"; tail -5 $O/ktrace_cfg5.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_rows -o run -- python3 tools/run_rows.py > $O/rows.json 2> $O/rows.err || { echo "ktrace rows failed"; tail -5 $O/rows.err; exit 1; }
./tools/pmc2.sh $O/pmc "--no-cfg5" > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
BPL=$(python3 -c "import json;print(json.load(open('$O/ktrace.json'))['roofline']['bytes_per_launch'])") || exit 1
python3 tools/pmc_traffic.py $O/pmc/summary.json $BPL tile_kernel $O/pmc_summary.json > $O/pmc_traffic.json || exit 1
echo done
