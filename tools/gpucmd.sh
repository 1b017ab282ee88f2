# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do for v in sp0 sp1; do
  PSG_LIB_PATH=$PWD/build/$v/libpsg.so timeout -k 10 300 python3 tools/shard_probe.py 30 > $O/sh_$v.txt 2> $O/sh_$v.err || { echo FAIL $v; tail -5 $O/sh_$v.err; exit 1; }
  echo "$rep $v $(cat $O/sh_$v.txt)"
done; done
bash tools/ab_run.sh "sp0 sp1" "cfg5" > $O/ab_split.txt 2>&1 || { echo AB FAILED; tail -5 $O/ab_split.txt; exit 1; }
cat $O/ab_split.txt
echo done
