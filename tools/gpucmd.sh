# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
R=r04; O=gpurun_out/$R; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/bench.json'));r=d['roofline']
print('cfg2 %.3e ms %.4f kern %.4f part %.4f frac %.3f step %.3f'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['partition_ms'],r['frac'],r['step_frac']))
print('f64', json.dumps(d.get('f64'))[:300])
print('cfg5', json.dumps(d.get('cfg5'))[:600])
print('rows', json.dumps({k:(v.get('ms'),v.get('frac')) for k,v in d.get('rows',{}).items()}))
print('e2e', json.dumps({k:v.get('value') for k,v in d.get('end_to_end',{}).items()}))
print('cpu', json.dumps(d.get('cpu_baseline')))
"
echo done
