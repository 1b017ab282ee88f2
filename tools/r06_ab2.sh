# r06 persistent-form A/B: default vs persistent vs persistent + start stagger
set -o pipefail
O=gpurun_out/${1:-r06f}; mkdir -p $O
for r in 1 2; do
for f in base pers runs; do
case $f in base) E=""; F=0;; pers) E=""; F=0x4000000;; *) E="PSG_LIB_PATH=build/$f/libpsg.so"; F=0x4000000;; esac
env $E timeout -k 10 120 python bench.py --profile-steps 1 --steps 40 --warmup 5 --plan-flags $F > $O/ab_${r}_$f.log 2>&1 || { tail -5 $O/ab_${r}_$f.log; exit 1; }
echo "$r $f $(grep 'profile run' $O/ab_${r}_$f.log)"
done; done
