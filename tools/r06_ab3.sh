# r06 search-window A/B: shipped (read2_b64 window, lazy bucket end) vs aligned 16-B window vs r05 HEAD build
set -o pipefail
O=gpurun_out/${1:-r06h}; mkdir -p $O
PSG_LIB_PATH=build/win128/libpsg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "cfg2 or random or nan or corner or extreme or cfg3" > $O/win128_test.log 2>&1 || { tail -30 $O/win128_test.log; exit 1; }
tail -1 $O/win128_test.log
for r in 1 2 3; do
for f in r05 cur win128; do
env PSG_LIB_PATH=build/$f/libpsg.so timeout -k 10 120 python bench.py --profile-steps 1 --steps 40 --warmup 5 > $O/ab_${r}_$f.log 2>&1 || { tail -5 $O/ab_${r}_$f.log; exit 1; }
echo "$r $f $(grep 'profile run' $O/ab_${r}_$f.log)"
done; done
