#!/bin/bash
# GPU box: rocprofv3 counters of the aggregate and partition kernels, one
# counter group per pass (MI355X_MICROARCH.md: no pass splitting; at most
# 8 SQ / 4 TCC counters per pass).  usage:
#   tools/pmc2.sh <outdir> "<bench args>"      PASSES="1 2 3" limits the groups
set -o pipefail
export TMPDIR=/tmp
OUT=$1
BARGS=${2:-}
mkdir -p $OUT
BENCH="python3 bench.py --profile-steps 1 --steps 3 --warmup 1 --no-cpu-baseline --no-check $BARGS"
ALL=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" \
     "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
     "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC" \
     "SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAVES" \
     "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_BUSY_CYCLES" \
     "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE")
for i in ${PASSES:-1 2 3 4 5 6 7 8 9}; do
  grp=${ALL[$((i-1))]}
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- $BENCH > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.json
echo done
