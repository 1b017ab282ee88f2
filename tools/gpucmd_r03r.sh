# session re-entry: GPU tests + side lines on the committed build; cfg2 2048-slot-tile A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03r; mkdir -p $O
WLS="cfg2 cfg3 cfg4 cfg5" bash tools/quick_bench.sh $O || exit 1
for f in 0x20000 0 0x20000 0; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cfg5 --steps 20 --plan-flags $f > $O/ab.json 2> $O/ab.err || { echo "ab failed"; tail -3 $O/ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab.json'));r=d['roofline'];print('[$f] cfg2 kern %.4f part %.4f frac %.3f step %.4f'%(r['kernel_ms'],r['partition_ms'],r['frac'],d['ms_per_step']))" | tee -a $O/ab.txt
done
for L in separate arena; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg5 --steps 10 --layout $L > $O/l5.json 2> $O/l5.err || { echo "layout failed"; tail -3 $O/l5.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/l5.json'));r=d['roofline'];print('[$L] cfg5 kern %.4f part %.4f frac %.3f step %.4f'%(r['kernel_ms'],r['partition_ms'],r['frac'],d['ms_per_step']))" | tee -a $O/ab.txt
done
