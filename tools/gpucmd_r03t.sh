# slabs in the context pool (cfg5 through psg_push: merge kernel time), arena-size A/B (plan API)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03t; mkdir -p $O
for v in noslab slab; do
  PSG_LIB_PATH=$PWD/build/$v/libpsg.so timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/srv_$v -o run -- python3 tools/run_cfg5_server.py 3 > $O/srv_$v.json 2> $O/srv_$v.err || { echo "srv $v failed"; tail -5 $O/srv_$v.err; exit 1; }
  echo "== $v $(cat $O/srv_$v.json)"
  grep -h "tile_packed\|partition_kernel" $(find $O/srv_$v -name "*kernel_stats.csv") | cut -d, -f1-4 | tee -a $O/ab.txt
done
for K in 0 64 16 4; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg5 --steps 10 --arena-pushes $K > $O/l5.json 2> $O/l5.err || { echo "arena $K failed"; tail -3 $O/l5.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/l5.json'));r=d['roofline'];print('[arena-pushes $K] cfg5 kern %.4f part %.4f frac %.3f step %.4f'%(r['kernel_ms'],r['partition_ms'],r['frac'],d['ms_per_step']))" | tee -a $O/ab.txt
done
