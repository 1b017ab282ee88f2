#!/bin/bash
# GPU box: counters of the SURVEY 8(f) row kernels (tools/run_rows.py), one
# group per rocprofv3 --pmc pass: what bounds gather, CountMin, snappy, the
# N-way merge and Darling.  usage: [ROWS="countmin snappy"] tools/pmc_rows.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
OUT=$1
mkdir -p $OUT
ALL=("FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
     "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
     "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" \
     "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVES")
for i in ${PASSES:-1 2 3 4 5 6}; do
  grp=${ALL[$((i-1))]}
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 tools/run_rows.py ${ROWS:-} > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT > $OUT/summary.json
echo done
