# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
for rep in 1 2; do for v in r16 r4 r1; do
  PSG_LIB_PATH=$PWD/build/$v/libpsg.so timeout -k 10 300 python3 tools/nway_probe.py > $O/nw_$v.txt 2>&1 || { echo FAIL $v; tail -5 $O/nw_$v.txt; exit 1; }
  echo "$rep $v $(grep batch $O/nw_$v.txt | tail -1)"
done; done
echo done
