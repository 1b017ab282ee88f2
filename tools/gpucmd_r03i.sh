# push-arena input layout A/B (bench --arena) on cfg2 / cfg3 / cfg5
mkdir -p gpurun_out/r03i
for a in "" "--arena" "" "--arena"; do
  for w in cfg2 cfg3 cfg5; do
    wa="--workload $w"; [ $w = cfg2 ] && wa="--no-cfg5"
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-check $wa --steps 10 $a > gpurun_out/r03i/ab.json 2> gpurun_out/r03i/ab.err || { echo FAIL; tail -3 gpurun_out/r03i/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/r03i/ab.json'));r=d['roofline'];print('[$a] $w kern %.4f part %.4f frac %.3f'%(r['kernel_ms'],r['partition_ms'],r['frac']))"
  done
done
