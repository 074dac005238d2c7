set -u
# r05q: band residual kernel with fewer VALU per node (no per-row lane masks, Dirichlet data linear in the row,
# three accumulators): residual / flux parity tests, then the residual bench (no CPU leg)
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05q}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k "cgr or flux or residual or vo" --timeout 120 --timeout-method thread > $OUT/${T}_tests.log 2>&1
rc=$?; tail -2 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/residual_bench.py $OUT/${T}_residual.json --no-cpu > $OUT/${T}_residual.log 2>&1
rc=$?; cat $OUT/${T}_residual.log | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['grid'], d['flux'], d['us_per_launch'], d['roofline']['frac'])"
exit $rc
