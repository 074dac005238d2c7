set -u
# r05r: the flux diagonal term per row (drow) / at the band's end (dend) / default (end for r <= 8):
# flux parity tests on the default, then the residual bench per arm (no CPU leg)
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05r}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "cgr or flux or residual or vo" --timeout 120 --timeout-method thread > $OUT/${T}_tests.log 2>&1
rc=$?; tail -2 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
for arm in - pf8 pf16; do
  if [ "$arm" = "-" ]; then unset GPI_LIB_VARIANT; else export GPI_LIB_VARIANT=$arm; fi
  timeout -k 10 300 python -u tools/residual_bench.py $OUT/${T}_residual_$arm.json --no-cpu > $OUT/${T}_residual_$arm.log 2>&1
  rc=$?; echo "arm $arm"; cat $OUT/${T}_residual_$arm.log | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['grid'], d['flux'], d['us_per_launch'], d['roofline']['frac'])"
  [ $rc -eq 0 ] || exit $rc
done
