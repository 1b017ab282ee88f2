# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/ab_run.sh "fu0 dd0 dd1" "cfg2 cfg3" > $O/ab_ddma.txt 2>&1 || { echo AB FAILED; tail -5 $O/ab_ddma.txt; exit 1; }
cat $O/ab_ddma.txt
for rep in 1 2; do for v in sn64 sn16 sn8; do
  PSG_LIB_PATH=$PWD/build/$v/libpsg.so timeout -k 10 300 python3 tools/run_rows.py snappy > $O/sn_$v.json 2> $O/sn_$v.err || { echo FAIL $v; tail -5 $O/sn_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sn_$v.json'));print('$rep $v', ' '.join('%s %.3f ms %.1f GB/s'%(k,x['ms'],x['GBps']) for k,x in d.items()))"
done; done
echo done
