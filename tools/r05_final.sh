#!/bin/bash
# Round-5 record at HEAD (GPU box, repo root): the GPU test suite as the driver runs it, smoke, the default
# bench line (CPU baseline + roofline), and a rocprofv3 kernel trace of a short bench run (kernel stats and
# the per-step timeline; traced at one step per graph replay, so the timeline splits into steps).  Every GPU step has its own time limit; stops at the first failing step.
# usage: tools/r05_final.sh TAG
set -u
TAG=${1:-r05z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$OUT/gpu_tests_$TAG.log" 2>&1
rc=$?; tail -2 "$OUT/gpu_tests_$TAG.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; tail -2 "$OUT/smoke_$TAG.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.log"
rc=$?; tail -1 "$OUT/bench_$TAG.json"; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --unroll 1 --no-cpu-baseline --no-roofline > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R"
python3 tools/prof_summary.py "$OUT/prof_$TAG" > "$OUT/kstats_$TAG.txt" 2>&1
python3 tools/step_timeline.py "$OUT/prof_$TAG" > "$OUT/timeline_$TAG.txt" 2>&1
tail -3 "$OUT/timeline_$TAG.txt"
exit 0
