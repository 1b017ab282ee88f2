# MEASUREMENT AID: cfg3 side line under knob settings (GPU box)
set -o pipefail
for v in ${KNOBS:-"PSG_WIDE=0" "PSG_WIDE=1"}; do
  echo "== $v"
  env $v timeout -k 10 300 python3 bench.py --workload cfg3 --no-cpu-baseline --steps 20 $ARGS > gpurun_out/ab3.json 2> gpurun_out/ab3.err || { tail -3 gpurun_out/ab3.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab3.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms'], r['partition_ms'], r['frac'], r['step_frac'])"
done
