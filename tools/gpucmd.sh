# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_run.sh "dd0 dd1" "cfg2 cfg5" > $O/ab_ddma.txt 2>&1 || { echo AB FAILED; tail -5 $O/ab_ddma.txt; exit 1; }
cat $O/ab_ddma.txt
timeout -k 10 300 python3 tools/run_rows.py snappy countmin > $O/rows.json 2> $O/rows.err || { echo ROWS FAILED; tail -5 $O/rows.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rows.json'));[print(k,'%.3f ms %.1f GB/s'%(x['ms'],x['GBps'])) for k,x in d.items()]"
timeout -k 10 300 python3 tools/pipe_probe.py cfg2 1 2 4 > $O/pipe_cfg2.txt 2> $O/pipe.err || { echo PIPE FAILED; tail -5 $O/pipe.err; exit 1; }
cat $O/pipe_cfg2.txt
timeout -k 10 400 python3 tools/pipe_probe.py cfg5 1 2 > $O/pipe_cfg5.txt 2>> $O/pipe.err || { echo PIPE5 FAILED; tail -5 $O/pipe.err; exit 1; }
cat $O/pipe_cfg5.txt
timeout -k 10 300 python3 tools/e2e/run_e2e.py 7 > $O/e2e.json 2> $O/e2e.err || { echo E2E FAILED; tail -5 $O/e2e.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/e2e.json'));[print(k, json.dumps(v)[:200]) for k,v in d.items()]"
echo done
