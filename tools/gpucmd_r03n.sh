# dense pushes through psg_push: pinned keys checked in place; cfg4 server-API device time
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03n; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread -k "pinned_keys" > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/cfg4srv -o run -- python3 tools/run_cfg4_server.py --pageable-out > $O/cfg4srv.json 2> $O/cfg4srv.err || { echo "cfg4srv failed"; tail -5 $O/cfg4srv.err; exit 1; }
cat $O/cfg4srv.json
timeout -k 10 400 python3 bench.py --no-cpu-baseline --workload cfg4 --steps 10 > $O/cfg4.json 2> $O/cfg4.err || { echo "cfg4 failed"; tail -5 $O/cfg4.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg4.json'));r=d['roofline'];print('cfg4 plan kern %.4f frac %.3f'%(r['kernel_ms'],r['frac']));print(json.dumps(d.get('server_api')))"
find $O/cfg4srv -name "*kernel_stats.csv" | head -1 | xargs cat
