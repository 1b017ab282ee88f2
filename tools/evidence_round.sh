# A round's final evidence: GPU tests, smoke, profile_round, side lines, row counters.  usage: tools/evidence_round.sh r04
set -o pipefail
export TMPDIR=/tmp
R=${1:-r04}; O=gpurun_out/$R; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKEFAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile_round.sh $R > $O/profile_round.log 2>&1 || { echo PROFFAIL; tail -20 $O/profile_round.log; exit 1; }
NOTEST=1 WLS="cfg3 cfg4" bash tools/quick_bench.sh $O/side || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cfg5 --dtype f64 > $O/side/cfg2_f64.json 2> $O/side/cfg2_f64.err || { echo "f64 failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/side/cfg2_f64.json'));r=d['roofline'];print('cfg2 f64 %.3e kern %.4f part %.4f frac %.3f step_frac %.3f'%(d['value'],r['kernel_ms'],r['partition_ms'],r['frac'],r['step_frac']))"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg5 --layout separate > $O/side/cfg5_separate.json 2> $O/side/cfg5_separate.err || { echo "cfg5 separate failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/side/cfg5_separate.json'));r=d['roofline'];print('cfg5 separate kern %.4f part %.4f frac %.3f'%(r['kernel_ms'],r['partition_ms'],r['frac']))"
bash tools/pmc_rows.sh $O/pmc_rows > $O/pmc_rows.log 2>&1 || { echo "pmc rows failed"; tail -5 $O/pmc_rows.log; exit 1; }
echo done
