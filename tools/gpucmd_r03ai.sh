# per-wave collision bitmaps in the context path too (bucket table rebuilt when another pass follows):
# GPU tests, cfg5 through psg_push (merge kernel time), cfg5 plan line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ai; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/srv -o run -- python3 tools/run_cfg5_server.py 3 > $O/srv.json 2> $O/srv.err || { echo "srv failed"; tail -5 $O/srv.err; exit 1; }
python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/srv/**/*kernel_stats.csv',recursive=True)[0])):
  if 'tile_packed' in r['Name'] or 'partition_kernel' in r['Name']: print(r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, 'us')
"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg5 > $O/cfg5.json 2> $O/cfg5.err || { echo "cfg5 failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg5.json'));r=d['roofline'];print('cfg5 plan kern %.4f part %.4f frac %.3f'%(r['kernel_ms'],r['partition_ms'],r['frac']))"
