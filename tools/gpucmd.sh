# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_freq_filter.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/test_freq.log 2>&1 || { echo FREQ FAILED; tail -30 $O/test_freq.log; exit 1; }
tail -3 $O/test_freq.log
timeout -k 10 300 python3 tools/run_rows.py > $O/rows.json 2> $O/rows.err || { echo ROWS FAILED; tail -5 $O/rows.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rows.json'));[print(k,json.dumps(v)[:300]) for k,v in d.items()]" || true
bash tools/ab_run.sh "sk0 sk4k sk8k sk20k fu0 fu4k fu8k fu20k" "cfg2" > $O/ab_occ.txt 2>&1 || { echo AB FAILED; tail -5 $O/ab_occ.txt; exit 1; }
cat $O/ab_occ.txt
timeout -k 10 600 python3 -u -m pytest tests/test_exchange_gpu.py -k full_cfg5 -x -v --timeout 600 --timeout-method thread > $O/test_full_cfg5.log 2>&1 || { echo FULLCFG5 FAILED; tail -30 $O/test_full_cfg5.log; exit 1; }
tail -3 $O/test_full_cfg5.log
echo done
