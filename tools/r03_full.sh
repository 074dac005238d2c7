#!/bin/bash
# full GPU test suite + ROM probe + bench (one GPU call); every step bounded, stop on a hard failure
set -u
TAG=${1:-r03}
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/t_$TAG.log 2>&1
rc=$?; tail -3 $OUT/t_$TAG.log; [ $rc -ne 0 ] && exit $rc
GPI_LIB_VARIANT=timing timeout -k 10 120 python tools/rom_probe.py 50 > $OUT/rom_$TAG.txt 2>&1 || exit $?
tail -3 $OUT/rom_$TAG.txt
timeout -k 10 300 python bench.py --steps 300 --warmup 100 --no-cpu-baseline --kprof $OUT/kprof_$TAG.json > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.log || exit $?
cat $OUT/bench_$TAG.json
