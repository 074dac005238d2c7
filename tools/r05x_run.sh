set -u
# r05x: MFMA input gradient by pixel-block pairs (GPI_IG_PAIR=1 build 'pair') vs the default: the codec / C64
# parity tests on the pair build, interleaved A/B, rocprof kernel stats of the pair arm
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05x}
GPI_LIB_VARIANT=pair timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c64.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/${T}_tests.log 2>&1
rc=$?; tail -2 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
ITER_TESTS=none ITER_REPS=3 ITER_STEPS=400 ITER_PROF=0 bash tools/r04_iter.sh ${T}_ab - GPI_LIB_VARIANT=pair || exit 1
cd /tmp && export TMPDIR=/tmp
for arm in "pair"; do
  export GPI_LIB_VARIANT=$arm
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${T}_$arm" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/prof_${T}_$arm.log" 2>&1
  rc=$?; echo "rocprof [$arm] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 $R/tools/prof_summary.py "$OUT/prof_${T}_$arm" 60 | grep -i "conv_bwd" | head -20
done
