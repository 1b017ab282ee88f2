# r06 tile-kernel form A/B (one box): form tests, then default vs persistent vs staged
set -o pipefail
O=gpurun_out/${1:-r06d}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_tile_forms_gpu.py -x -q --timeout 200 --timeout-method thread > $O/forms_test.log 2>&1 || { tail -30 $O/forms_test.log; exit 1; }
tail -2 $O/forms_test.log
for r in 1 2; do
for f in 0 0x4000000 0x1000000; do
timeout -k 10 120 python bench.py --profile-steps 1 --steps 40 --warmup 5 --plan-flags $f > $O/ab_${r}_$f.log 2>&1 || { tail -5 $O/ab_${r}_$f.log; exit 1; }
echo "$r $f $(grep 'profile run' $O/ab_${r}_$f.log)"
done; done
