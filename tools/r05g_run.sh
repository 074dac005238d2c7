set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05g}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 460 --timeout-method thread > $OUT/${T}_tests.log 2>&1
rc=$?; tail -4 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
ITER_TESTS=none ITER_REPS=2 ITER_STEPS=400 ITER_PROF=0 bash tools/r04_iter.sh ${T}_ab - GPI_LIB_VARIANT=novdg3
for arm in "GPI_LIB_VARIANT=pf2" "GPI_LIB_VARIANT=pf6" "-"; do
  E=""; [ "$arm" = "-" ] || E="$arm"
  env $E timeout -k 10 200 python -u tools/residual_bench.py > $OUT/${T}_res_$(echo $arm | tr = _).log 2>&1
  rc=$?; echo "residual [$arm] rc=$rc"; grep '"flux"' $OUT/${T}_res_$(echo $arm | tr = _).log | cut -c1-110; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python -u bench.py --kprof $OUT/${T}_kprof.json --steps 50 --warmup 20 > $OUT/${T}_kprof_bench.json 2> $OUT/${T}_kprof.err; echo "kprof rc=$?"
GPI_LIB_VARIANT=novdg3 timeout -k 10 200 python -u bench.py --kprof $OUT/${T}_kprof_novdg3.json --steps 50 --warmup 20 > $OUT/${T}_kprof_novdg3_bench.json 2> $OUT/${T}_kprof_novdg3.err; echo "kprof novdg3 rc=$?"
