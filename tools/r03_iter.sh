set -u
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_c64.py tests/test_gpu_parity.py -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t_r03b.log 2>&1
rc=$?; tail -3 $OUT/t_r03b.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/phase_probe.py LastTransUp > $OUT/phase_r03b.txt 2>&1 || exit $?
cat $OUT/phase_r03b.txt
timeout -k 10 300 python bench.py --steps 300 --warmup 100 --no-cpu-baseline --kprof $OUT/kprof_r03b.json > $OUT/bench_r03b.json 2> $OUT/bench_r03b.log || exit $?
cat $OUT/bench_r03b.json
