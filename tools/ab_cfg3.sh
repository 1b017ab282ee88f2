# MEASUREMENT AID: cfg3 side line under kernel-form overrides (GPU box);
# FLAGS: include/psg.h values, e.g. 0x10000 (PSG_GROUP32) 0x20000 (PSG_GROUP64)
set -o pipefail
for f in ${FLAGS:-0x10000 0x20000}; do
  echo "== plan flags $f"
  timeout -k 10 300 python3 bench.py --workload cfg3 --no-cpu-baseline --steps 20 --plan-flags $f $ARGS > gpurun_out/ab3.json 2> gpurun_out/ab3.err || { tail -3 gpurun_out/ab3.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab3.json'));r=d['roofline'];print(d['value'], d['ms_per_step'], r['kernel'], r['kernel_ms'], r['partition_ms'], r['frac'], r['step_frac'])"
done
