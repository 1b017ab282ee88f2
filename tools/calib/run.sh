#!/bin/bash
# GPU box: FETCH_SIZE / WRITE_SIZE per byte for 4/8/16-B lane reads.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/calib
mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -shared -fPIC tools/calib/calib_fetch.hip -o tools/calib/libcalib.so || exit 1
i=0
for grp in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 tools/calib/calib_fetch.py > $OUT/p$i.log 2>&1 || { echo "calib pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
vals = collections.defaultdict(list)
for f in glob.glob("gpurun_out/calib/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        w = "16" if "u4" in n else ("8" if "unsigned long" in n or "uint64" in n or "mE" in n else "4")
        vals[(n[:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (n, c), v in sorted(vals.items()):
    m = sum(v) / len(v)
    extra = ""
    if c == "FETCH_SIZE":
        extra = "  -> bytes/(FETCH_SIZE*1024) = %.3f" % ((512 << 20) / (m * 1024))
    if c == "TCC_MISS_sum":
        extra = "  -> bytes/miss = %.1f" % ((512 << 20) / m)
    print(n, c, m, extra)
PY
