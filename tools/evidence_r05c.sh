# r05 evidence, part C: counters of the row kernels (CountMin, snappy, N-way, gather, crc, Darling).
set -o pipefail
export TMPDIR=/tmp
R=${1:-r05}; O=gpurun_out/$R; mkdir -p $O
bash tools/pmc_rows.sh $O/pmc_rows > $O/pmc_rows.log 2>&1 || { echo "pmc rows failed"; tail -5 $O/pmc_rows.log; exit 1; }
echo done
