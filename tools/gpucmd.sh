# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
R=r04; OUT=gpurun_out/$R; mkdir -p $OUT
PASSES="1 2 3 4 5 7" ./tools/pmc2.sh $OUT/pmc_cfg5 "--workload cfg5" > $OUT/pmc_cfg5.log 2>&1 || { echo "pmc cfg5 failed"; tail -5 $OUT/pmc_cfg5.log; exit 1; }
BPL5=$(python3 -c "import json;print(json.load(open('profiles/r04_bench.json'))['cfg5']['rank0']['bytes_per_launch'])") || exit 1
python3 tools/pmc_traffic.py $OUT/pmc_cfg5/summary.json $BPL5 tile_packed_kernel $OUT/pmc_summary_cfg5.json cfg5 > $OUT/pmc_traffic_cfg5.json || exit 1
echo pmc cfg5 ok
./tools/pmc_rows.sh $OUT/pmc_rows > $OUT/pmc_rows.log 2>&1 || { echo "pmc rows failed"; tail -5 $OUT/pmc_rows.log; exit 1; }
echo pmc rows ok
echo done
