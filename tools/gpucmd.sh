# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
R=r04; O=gpurun_out/$R; mkdir -p $O/side
NOTEST=1 WLS="cfg3 cfg4" bash tools/quick_bench.sh $O/side || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --workload cfg5 --layout separate > $O/side/cfg5_separate.json 2> $O/side/cfg5_separate.err || { echo "cfg5 separate failed"; exit 1; }
python3 -c "import json;d=json.load(open('$O/side/cfg5_separate.json'));r=d['roofline'];print('cfg5 separate kern %.4f part %.4f frac %.3f'%(r['kernel_ms'],r['partition_ms'],r['frac']))"
echo done
