# packed kernel: loads-and-stores skeleton vs the full kernel (cfg5)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03z; mkdir -p $O
bash tools/ab_run.sh "pk pkskel pkskel2" "cfg5" 2>&1 | tee $O/ab.txt
