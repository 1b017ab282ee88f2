#!/bin/bash
# GPU box: the round's committed evidence.  usage: tools/profile_round.sh r01
#   ktrace/      rocprofv3 --kernel-trace --stats of a bench run (default config)
#   pmc/         FETCH_SIZE / WRITE_SIZE / TCC passes (tools/pmc2.sh), one pass each
#   pmc_summary.json  HBM bytes per aggregate launch (read by bench.py as roofline.traffic)
#   bench.json   default bench line (N=1, with end-to-end + CPU baseline)
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
R=${1:-r01}
K=${PSG_KERNEL:-11}
OUT=gpurun_out/$R
mkdir -p $OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o run -- python3 bench.py --no-cpu-baseline > $OUT/ktrace.json 2> $OUT/ktrace.err || { echo "ktrace failed"; tail -5 $OUT/ktrace.err; exit 1; }
cat $OUT/ktrace.json
BPL=$(python3 -c "import json;print(json.load(open('$OUT/ktrace.json'))['roofline']['bytes_per_launch'])") || exit 1
PASSES="1 2 3" ./tools/pmc2.sh "$K:S" > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
rm -rf $OUT/pmc && mv gpurun_out/pmc2/k${K}S $OUT/pmc
python3 tools/pmc_traffic.py $OUT/pmc/summary.json $BPL tile_kernel profiles/pmc_summary.json > $OUT/pmc_traffic.json || exit 1
cp profiles/pmc_summary.json $OUT/pmc_summary.json
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo done
