# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo BENCHFAIL; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('value %.4e kern %.4f part %.4f frac %.3f step %.3f'%(d['value'],r['kernel_ms'],r['partition_ms'],r['frac'],r['step_frac']));print(' '.join('%s %.3f'%(k,v['ms_per_aggregate']) for k,v in d['end_to_end']['modes'].items()))"
echo done
