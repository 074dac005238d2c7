set -u
# r05ad: row-image staging with the chunk source by one select (GPI_STAGE_SEL=1, default) vs the compiler's branchy form (build branchy)
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05ad}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/${T}_tests.log 2>&1
rc=$?; tail -2 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
ITER_TESTS=none ITER_REPS=3 ITER_STEPS=400 ITER_PROF=0 bash tools/r04_iter.sh ${T}_ab - "GPI_LIB_VARIANT=branchy" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${T}" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/prof_${T}.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 $R/tools/prof_summary.py "$OUT/prof_${T}" 60 | grep -i "conv_" | head -30
GPI_LIB_VARIANT=branchy timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${T}_branchy" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/prof_${T}_branchy.log" 2>&1
rc=$?; echo "rocprof branchy rc=$rc"; [ $rc -eq 0 ] || exit $rc
