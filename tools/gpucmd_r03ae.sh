# packed kernel without the scratch spill: GPU tests, cfg5 kernel trace + traffic passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ae; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > $O/gputest.log 2>&1 || { echo TESTFAIL; tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_cfg5 -o run -- python3 bench.py --no-cpu-baseline --workload cfg5 > $O/ktrace_cfg5.json 2> $O/ktrace_cfg5.err || { echo "ktrace cfg5 failed"; tail -5 $O/ktrace_cfg5.err; exit 1; }
BPL5=$(python3 -c "import json;print(json.load(open('$O/ktrace_cfg5.json'))['roofline']['bytes_per_launch'])") || exit 1
PASSES="1 2 3" ./tools/pmc2.sh $O/pmc_cfg5 "--workload cfg5" > $O/pmc_cfg5.log 2>&1 || { echo "pmc cfg5 failed"; tail -5 $O/pmc_cfg5.log; exit 1; }
python3 tools/pmc_traffic.py $O/pmc_cfg5/summary.json $BPL5 tile_packed_kernel $O/pmc_summary_cfg5.json cfg5 > $O/pmc_traffic_cfg5.json || exit 1
python3 -c "import json;d=json.load(open('$O/ktrace_cfg5.json'));r=d['roofline'];print('cfg5 kern %.4f part %.4f frac %.3f step_frac %.3f'%(r['kernel_ms'],r['partition_ms'],r['frac'],r['step_frac']));p=json.load(open('$O/pmc_summary_cfg5.json'));print('traffic', p['ratio_to_algorithmic'], p['write_bytes'])"
