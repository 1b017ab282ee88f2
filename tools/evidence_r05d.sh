# r05 evidence, part D (final code): GPU tests, smoke, kernel traces of the
# default bench and of the rows, the final default bench line.
# usage: tools/evidence_r05d.sh r05d
set -o pipefail
export TMPDIR=/tmp
R=${1:-r05d}; O=gpurun_out/$R; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- python3 bench.py --no-cpu-baseline > $O/ktrace.json 2> $O/ktrace.err || { echo "ktrace failed"; tail -5 $O/ktrace.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_rows -o run -- python3 tools/run_rows.py > $O/rows.json 2> $O/rows.err || { echo "ktrace rows failed"; tail -5 $O/rows.err; exit 1; }
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench %.4e ms %.4f kern %.4f frac %.3f step %.3f'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['step_frac']))"
echo done
