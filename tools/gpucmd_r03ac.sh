# packed kernel on 4096-slot tiles (A/B build) vs 2048; GPU tests on the in-tree build (index API per tile size)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ac; mkdir -p $O
bash tools/ab_run.sh "ts2048 ts1024" "cfg5" 2>&1 | tee $O/ab.txt
