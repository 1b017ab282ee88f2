# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_freq_filter.py -x -v -m gpu --timeout 200 --timeout-method thread > $O/gputest_ff.log 2>&1 || { echo TESTFAIL; tail -40 $O/gputest_ff.log; exit 1; }
tail -2 $O/gputest_ff.log
timeout -k 10 300 python3 tools/run_rows.py > $O/rows.json 2> $O/rows.err || { echo ROWSFAIL; tail -5 $O/rows.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rows.json'));[print(k,'%.4f ms frac %.3f'%(v['ms'],v['frac'])) for k,v in d.items() if 'countmin' in k]"
bash tools/ab_run.sh "base skel base_o6 skel_o6 base_o4 skel_o4" "cfg2" 2>&1 | tee $O/ab_occ.txt
echo done
