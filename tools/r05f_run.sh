set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05f}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "cgr or flux or residual or vo" > $OUT/${T}_tests.log 2>&1
rc=$?; tail -4 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
for arm in "-" "GPI_CGR_FORM=1" "GPI_CGR_PF=4"; do
  E=""; [ "$arm" = "-" ] || E="$arm"
  if [ "$arm" = "GPI_CGR_PF=4" ]; then E="GPI_LIB_VARIANT=pf4"; fi
  env $E timeout -k 10 200 python -u tools/residual_bench.py > $OUT/${T}_res_$(echo $arm | tr = _).log 2>&1
  rc=$?; echo "residual [$arm] rc=$rc"; grep '"flux"' $OUT/${T}_res_$(echo $arm | tr = _).log | cut -c1-110; [ $rc -eq 0 ] || exit $rc
done
