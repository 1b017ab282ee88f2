# cfg3 traffic and SQ counters on the final build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03al; mkdir -p $O
timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg3 > $O/cfg3.json 2> $O/cfg3.err || { echo "cfg3 failed"; exit 1; }
BPL=$(python3 -c "import json;print(json.load(open('$O/cfg3.json'))['roofline']['bytes_per_launch'])") || exit 1
PASSES="1 2 3 4 5 7" ./tools/pmc2.sh $O/pmc_cfg3 "--workload cfg3" > $O/pmc_cfg3.log 2>&1 || { echo "pmc cfg3 failed"; tail -5 $O/pmc_cfg3.log; exit 1; }
python3 tools/pmc_traffic.py $O/pmc_cfg3/summary.json $BPL tile_kernel $O/pmc_summary_cfg3.json cfg3 > $O/pmc_traffic_cfg3.json || exit 1
python3 -c "import json;p=json.load(open('$O/pmc_summary_cfg3.json'));print('cfg3 traffic', p['ratio_to_algorithmic'], p.get('partition_hbm_bytes_per_launch'))"
