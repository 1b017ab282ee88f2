# skeleton A/B (loads+stores only / +search) vs the full tile kernel; cfg3 PMC traffic
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03k; mkdir -p $O
for rep in 1 2; do
for lib in "" build/skel1/libpsg.so build/skel2/libpsg.so; do
  for w in cfg2 cfg3; do
    wa="--workload $w"; [ $w = cfg2 ] && wa="--no-cfg5"
    PSG_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-check $wa --steps 10 > $O/ab.json 2> $O/ab.err || { echo FAIL; tail -3 $O/ab.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab.json'));r=d['roofline'];print('[$lib] $w kern %.4f part %.4f frac %.3f bpl %d'%(r['kernel_ms'],r['partition_ms'],r['frac'],r['bytes_per_launch']))"
  done
done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg3 --steps 5 > $O/cfg3.json 2> $O/cfg3.err || { echo FAIL3; exit 1; }
BPL=$(python3 -c "import json;print(json.load(open('$O/cfg3.json'))['roofline']['bytes_per_launch'])") || exit 1
PASSES="1 2 3 7" ./tools/pmc2.sh $O/pmc_cfg3 "--workload cfg3" > $O/pmc_cfg3.log 2>&1 || { echo "pmc cfg3 failed"; tail -5 $O/pmc_cfg3.log; exit 1; }
python3 tools/pmc_traffic.py $O/pmc_cfg3/summary.json $BPL tile_kernel $O/pmc_summary_cfg3.json cfg3 || exit 1
echo done
