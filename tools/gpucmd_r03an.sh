# cfg5 SQ counters (wave cycles, waits, instruction mix, LDS) on the final build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03an; mkdir -p $O
PASSES="4 5 6 7 8 9" ./tools/pmc2.sh $O/pmc_cfg5 "--workload cfg5" > $O/pmc_cfg5.log 2>&1 || { echo "pmc cfg5 failed"; tail -5 $O/pmc_cfg5.log; exit 1; }
python3 -c "
import json;d=json.load(open('$O/pmc_cfg5/summary.json'))['counters']
for k in ('tile_packed_kernel','partition_kernel'):
  c=d[k]; print(k, 'wait/wave %.2f'%(c['SQ_WAIT_ANY']/c['SQ_WAVE_CYCLES']), 'bank/lds %.2f'%(c['SQ_LDS_BANK_CONFLICT']/max(1,c['SQ_LDS_IDX_ACTIVE'])), 'salu/valu %.2f'%(c['SQ_INSTS_SALU']/c['SQ_INSTS_VALU']), 'lds insts %.3g'%c['SQ_INSTS_LDS'], 'valu %.3g'%c['SQ_INSTS_VALU'])
"
