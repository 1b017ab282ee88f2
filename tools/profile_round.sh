#!/bin/bash
# GPU box: the round's committed evidence.  usage: tools/profile_round.sh r02
#   ktrace/          rocprofv3 --kernel-trace --stats of the default bench (cfg2)
#   ktrace_cfg5/     the same for --workload cfg5 (packed rounds, stream partition)
#   ktrace_rows/     the same for the SURVEY 8(f) rows block (tools/run_rows.py)
#   pmc/             cfg2 counters, one group per rocprofv3 --pmc pass (tools/pmc2.sh)
#   pmc_cfg5/        cfg5 FETCH_SIZE / WRITE_SIZE / TCC passes
#   pmc_summary.json HBM bytes per launch of the tile and partition kernels (cfg2;
#                    read by bench.py as roofline.traffic)
#   bench.json       the default bench line (N=1, end-to-end + CPU baseline)
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
R=${1:-r02}
OUT=gpurun_out/$R
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o run -- python3 bench.py --no-cpu-baseline > $OUT/ktrace.json 2> $OUT/ktrace.err || { echo "ktrace failed"; tail -5 $OUT/ktrace.err; exit 1; }
BPL=$(python3 -c "import json;print(json.load(open('$OUT/ktrace.json'))['roofline']['bytes_per_launch'])") || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace_cfg5 -o run -- python3 bench.py --no-cpu-baseline --workload cfg5 > $OUT/ktrace_cfg5.json 2> $OUT/ktrace_cfg5.err || { echo "ktrace cfg5 failed"; tail -5 $OUT/ktrace_cfg5.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace_rows -o run -- python3 tools/run_rows.py > $OUT/rows.json 2> $OUT/rows.err || { echo "ktrace rows failed"; tail -5 $OUT/rows.err; exit 1; }
./tools/pmc2.sh $OUT/pmc "--no-cfg5" > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
python3 tools/pmc_traffic.py $OUT/pmc/summary.json $BPL tile_kernel profiles/pmc_summary.json > $OUT/pmc_traffic.json || exit 1
cp profiles/pmc_summary.json $OUT/pmc_summary.json
PASSES="1 2 3" ./tools/pmc2.sh $OUT/pmc_cfg5 "--workload cfg5" > $OUT/pmc_cfg5.log 2>&1 || { echo "pmc cfg5 failed"; tail -5 $OUT/pmc_cfg5.log; exit 1; }
BPL5=$(python3 -c "import json;print(json.load(open('$OUT/ktrace_cfg5.json'))['roofline']['bytes_per_launch'])") || exit 1
python3 tools/pmc_traffic.py $OUT/pmc_cfg5/summary.json $BPL5 tile_packed_kernel profiles/pmc_summary_cfg5.json cfg5 > $OUT/pmc_traffic_cfg5.json || exit 1
cp profiles/pmc_summary_cfg5.json $OUT/pmc_summary_cfg5.json
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo done
