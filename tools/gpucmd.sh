# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d; mkdir -p $O
bash tools/ab_run.sh "base sk1 sk2 sk3 sk4 o6 o4 sk1o4" "cfg2" 2>&1 | tee $O/ab_phases.txt
echo done
