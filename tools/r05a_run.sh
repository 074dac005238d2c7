set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 460 --timeout-method thread --durations=20 > $OUT/r05a_tests.log 2>&1
rc=$?; tail -25 $OUT/r05a_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/r05a_bench.json 2> $OUT/r05a_bench.log
rc=$?; tail -1 $OUT/r05a_bench.json; [ $rc -eq 0 ] || exit $rc
bash tools/r05_counters.sh r05a
