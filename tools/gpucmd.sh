# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06t; mkdir -p $O
PSG_LIB_PATH=$PWD/build/sprof/libpsg.so timeout -k 10 120 python3 tools/snappy_prof.py > $O/sprof.json 2> $O/sprof.err || { echo SPROF FAILED; tail -5 $O/sprof.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/sprof.json'))
for n,v in d.items():
  print(n, 'ms', round(v['ms'],4))
  for p in v['per_part'][:2]: print('  ', p['bytes_in'], p['tab'])
"
bash tools/evidence_r06.sh r06e
