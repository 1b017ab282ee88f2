# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
bash tools/ab_run.sh "dd1 c8 c9" "cfg3" > $O/ab_cfg3.txt 2>&1 || { echo AB FAILED; tail -5 $O/ab_cfg3.txt; exit 1; }
cat $O/ab_cfg3.txt
echo done
