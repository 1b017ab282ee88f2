#!/bin/bash
# GPU box: kernel timings of A/B builds (build/<name>/libpsg.so), interleaved
# twice on the same box.  usage: tools/ab_run.sh "<name> <name> ..." "<workloads>"
O=gpurun_out/ab; mkdir -p $O
for rep in 1 2; do
for v in $1; do
  for w in ${2:-cfg2 cfg5}; do
    a="--workload $w"; [ $w = cfg2 ] && a="--no-cfg5"
    PSG_LIB_PATH=$PWD/build/$v/libpsg.so timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-check --no-f64 $a --steps 10 > $O/out.json 2> $O/err.log || { echo FAIL $v $w; tail -3 $O/err.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/out.json'));r=d['roofline'];print('$rep $v $w kern %.3f part %.3f'%(r['kernel_ms'],r['partition_ms']))"
  done
done
done
