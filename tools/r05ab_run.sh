set -u
# r05ab: fused output conv with the exp-field loss as its own instantiation (EXF; default build) vs the build of
# the previous commit (runtime flag, selects: 'prev', GPI_ALLOW_STALE_LIB=1): GPU suite, interleaved A/B, kernel stats
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05ab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/${T}_tests.log 2>&1
rc=$?; tail -2 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
ITER_TESTS=none ITER_REPS=3 ITER_STEPS=400 ITER_PROF=0 bash tools/r04_iter.sh ${T}_ab - "GPI_LIB_VARIANT=prev GPI_ALLOW_STALE_LIB=1" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${T}" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/prof_${T}.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 $R/tools/prof_summary.py "$OUT/prof_${T}" 60 | grep -i "conv_bwd_kernel<5" | head -4
