# scratch GPU command of the current step (overwritten per gpurun call)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_wire.py tests/test_nway_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "cursor or cfg2 or cfg5 or packed or partition or key_cache or signature or nway or union" > $O/gputest_cursor.log 2>&1 || { echo TESTFAIL; tail -40 $O/gputest_cursor.log; exit 1; }
tail -2 $O/gputest_cursor.log
summ() { python3 -c "import json,sys;d=json.load(open('$O/b.json'));r=d['roofline'];print(sys.argv[1],'value %.3e ms/step %.4f kern %.4f part %.4f frac %.3f step %.3f %s'%(d['value'],d['ms_per_step'],r['kernel_ms'],r['partition_ms'],r['frac'],r['step_frac'],r['kernel']))" "$1"; }
for rep in 1 2; do
for f in 0 0x800000; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cfg5 --no-f64 --steps 20 --plan-flags $f > $O/b.json 2> $O/b.err || { echo "bench failed $f"; tail -5 $O/b.err; exit 1; }
  summ "cfg2 $rep flags $f"
  timeout -k 10 300 python3 bench.py --workload cfg5 --steps 10 --plan-flags $f > $O/b.json 2> $O/b.err || { echo "bench cfg5 failed $f"; tail -5 $O/b.err; exit 1; }
  summ "cfg5 $rep flags $f"
done
done
echo done
