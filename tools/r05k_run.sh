set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05k}
cd /tmp && export TMPDIR=/tmp
for arm in "-" "vdg3"; do
  if [ "$arm" = "-" ]; then unset GPI_LIB_VARIANT; else export GPI_LIB_VARIANT=$arm; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${T}_$arm" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --unroll 1 --no-cpu-baseline --no-roofline > "$OUT/prof_${T}_$arm.log" 2>&1
  rc=$?; echo "rocprof [$arm] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 $R/tools/step_timeline.py "$OUT/prof_${T}_$arm" > "$OUT/timeline_${T}_$arm.txt" 2>&1
  tail -3 "$OUT/timeline_${T}_$arm.txt"
done
