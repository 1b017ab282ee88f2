# r06 snappy table form: tests, then A/B (table form vs the streamed form,
# PSG_SNAPPY_IR=1 build) on the e2e parts and the end-to-end compressed mode
set -o pipefail
O=gpurun_out/${1:-r06m}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_wire.py -x -q --timeout 200 --timeout-method thread -k "snappy or compress" > $O/snappy_test.log 2>&1 || { tail -30 $O/snappy_test.log; exit 1; }
tail -1 $O/snappy_test.log
for r in 1 2; do
for f in tab ir; do
if [ $f = ir ]; then E="PSG_LIB_PATH=build/snir1/libpsg.so"; else E=""; fi
env $E timeout -k 10 120 python tools/snappy_time.py > $O/parts_${r}_$f.json 2>&1 || { tail -5 $O/parts_${r}_$f.json; exit 1; }
echo "$r $f parts $(cat $O/parts_${r}_$f.json)"
env $E timeout -k 10 200 python tools/e2e/run_e2e.py 7 pinned,compressed > $O/e2e_${r}_$f.json 2>$O/e2e_${r}_$f.err || { tail -5 $O/e2e_${r}_$f.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('$O/e2e_${r}_$f.json')); print('$r $f e2e', {k: round(v['ms_per_aggregate'],4) for k,v in d['modes'].items()})"
done; done
