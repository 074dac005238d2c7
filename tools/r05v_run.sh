set -u
# r05v: FOM tests with the multigrid default (32^2+), then the FOM bench record with its CPU baseline
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05v}
timeout -k 10 400 python -u -m pytest tests/test_gpu_fom.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/${T}_tests.log 2>&1
rc=$?; tail -2 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/fom_bench.py --out $OUT/${T}_fom_bench.json > $OUT/${T}_fom.log 2>&1
rc=$?; cut -c1-220 $OUT/${T}_fom.log; exit $rc
