set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05i}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 460 --timeout-method thread > $OUT/${T}_tests.log 2>&1
rc=$?; tail -3 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
OPS="EncBlock1.denselayer1.conv1 DecBlock3.denselayer1.conv1 LastTransUp.conv1"
for arm in "-" "GPI_LIB_VARIANT=novdg3"; do
  E=""; [ "$arm" = "-" ] || E="$arm"
  env $E timeout -k 10 200 python -u tools/phase_probe.py $OPS > $OUT/${T}_phase_$(echo $arm | tr = _).txt 2>&1
  rc=$?; echo "== [$arm] rc=$rc"; grep -E "bwd blocks|cycles/phase" $OUT/${T}_phase_$(echo $arm | tr = _).txt; [ $rc -eq 0 ] || exit $rc
done
ITER_TESTS=none ITER_REPS=3 ITER_STEPS=400 ITER_PROF=0 bash tools/r04_iter.sh ${T}_ab - GPI_LIB_VARIANT=novdg3
