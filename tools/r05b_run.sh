set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05b}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 460 --timeout-method thread --durations=12 > $OUT/${T}_tests.log 2>&1
rc=$?; tail -16 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
for arm in "-" "GPI_CGR_STREAM=0" "GPI_LIB_VARIANT=d3"; do
  E=""; [ "$arm" = "-" ] || E="$arm"
  env $E timeout -k 10 200 python -u tools/residual_bench.py > $OUT/${T}_res_${arm%%=*}.log 2>&1
  rc=$?; echo "residual [$arm] rc=$rc"; grep '"flux"' $OUT/${T}_res_${arm%%=*}.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python bench.py > $OUT/${T}_bench.json 2> $OUT/${T}_bench.log
rc=$?; tail -1 $OUT/${T}_bench.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
bash tools/r05_counters.sh $T
