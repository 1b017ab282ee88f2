# the default bench line on the final build (what the driver runs), plus smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03aj; mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));r=d['roofline'];print('value %.4g ms/step %.4f kern %.4f frac %.3f step_frac %.3f'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'],r['step_frac']));c=d['cfg5'];print('cfg5', c['ms_per_step'], c['rank0']['kernel_ms'], c['modes']['unsliced'].get('ms_per_step'))"
