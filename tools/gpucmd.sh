# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_wire.py tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "snappy or compress or wire or cache" > $O/test_sn.log 2>&1 || { echo TESTFAIL; tail -30 $O/test_sn.log; exit 1; }
echo "tests $(tail -1 $O/test_sn.log)"
PSG_LIB_PATH=$PWD/build/sprof/libpsg.so timeout -k 10 300 python3 tools/snappy_prof.py > $O/sprof.json 2> $O/sprof.err || { echo FAIL; tail -5 $O/sprof.err; exit 1; }
python3 - <<'P'
import json
d=json.load(open('gpurun_out/ab/sprof.json'))
for k,v in d.items():
    print(k, 'ms %.3f'%v['ms'])
    for i,p in enumerate(v['per_part'][:2]):
        print(' ', i, p)
P
timeout -k 10 300 python3 tools/run_rows.py > $O/rows.json 2> $O/rows.err || { echo ROWSFAIL; tail -5 $O/rows.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/rows.json'));r=d.get('rows',d);[print(k,'%.4f ms'%r[k]['ms'],'frac %.3f'%r[k]['frac']) for k in r if 'snappy' in k]"
timeout -k 10 300 python3 tools/e2e/run_e2e.py 7 compressed,pinned > $O/e2e.json 2> $O/e2e.err || { echo E2EFAIL; tail -5 $O/e2e.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/e2e.json'));[print(k,v['ms_per_aggregate']) for k,v in d['modes'].items()]"
echo done
