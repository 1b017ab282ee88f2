# r05 evidence, part B: cfg5 PMC passes, the final default bench line, side lines.
set -o pipefail
export TMPDIR=/tmp
R=${1:-r05}; O=gpurun_out/$R; mkdir -p $O $O/side
# A/B of the once-written splitters (sp0 = before, sp1 = after): one cfg5 shard, the whole cfg5
if [ -d build/sp0 ] && [ -d build/sp1 ]; then
  for rep in 1 2; do for v in sp0 sp1; do
    PSG_LIB_PATH=$PWD/build/$v/libpsg.so timeout -k 10 300 python3 tools/shard_probe.py 30 > $O/sh_$v.txt 2> $O/sh_$v.err || { echo FAIL $v; tail -5 $O/sh_$v.err; exit 1; }
    echo "$rep $v $(cat $O/sh_$v.txt)" | tee -a $O/ab_split.txt
  done; done
  bash tools/ab_run.sh "sp0 sp1" "cfg5" >> $O/ab_split.txt 2>&1 || { echo AB FAILED; tail -5 $O/ab_split.txt; exit 1; }
  tail -4 $O/ab_split.txt
fi
# the packed kernel's memory side alone (PSG_SKELETON=1: loads and stores, no search or fold)
if [ -d build/pks ]; then
  bash tools/ab_run.sh "sp1 pks" "cfg5" > $O/ab_packed_skeleton.txt 2>&1 || { echo AB FAILED; tail -5 $O/ab_packed_skeleton.txt; exit 1; }
  cat $O/ab_packed_skeleton.txt
fi
PASSES="1 2 3" ./tools/pmc2.sh $O/pmc_cfg5 "--workload cfg5" > $O/pmc_cfg5.log 2>&1 || { echo "pmc cfg5 failed"; tail -5 $O/pmc_cfg5.log; exit 1; }
timeout -k 10 600 python3 bench.py --no-cpu-baseline --workload cfg5 --steps 5 > $O/cfg5_bpl.json 2> $O/cfg5_bpl.err || exit 1
BPL5=$(python3 -c "import json;print(json.load(open('$O/cfg5_bpl.json'))['roofline']['bytes_per_launch'])") || exit 1
python3 tools/pmc_traffic.py $O/pmc_cfg5/summary.json $BPL5 tile_packed_kernel $O/pmc_summary_cfg5.json cfg5 > $O/pmc_traffic_cfg5.json || exit 1
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('bench %.4e ms %.4f kern %.4f frac %.3f step %.3f'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['step_frac']))"
NOTEST=1 WLS="cfg3 cfg4" bash tools/quick_bench.sh $O/side || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cfg5 --dtype f64 > $O/side/cfg2_f64.json 2> $O/side/cfg2_f64.err || { echo "f64 failed"; exit 1; }
echo done
