#!/bin/bash
# One GPU pass: parity tests -> smoke -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; anything but a clean exit / ordinary
# test failure (rc 0 or 1) ends the script before the next GPU step.
# usage: tools/gpu_round.sh [tag] [bench args...]
set -u
TAG=${1:-r01}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"

timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > "$OUT/gpu_tests_$TAG.log" 2>&1
rc=$?
echo "pytest rc=$rc" >> "$OUT/gpu_tests_$TAG.log"
tail -5 "$OUT/gpu_tests_$TAG.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after pytest rc=$rc"; exit $rc; fi

timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?
tail -3 "$OUT/smoke_$TAG.log"
if [ $rc -ne 0 ]; then echo "stop after smoke rc=$rc"; exit $rc; fi

timeout -k 10 400 python bench.py "$@" > "$OUT/bench_$TAG.log" 2>&1
rc=$?
tail -2 "$OUT/bench_$TAG.log"
if [ $rc -ne 0 ]; then echo "stop after bench rc=$rc"; exit $rc; fi

cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/prof_$TAG.log" 2>&1
rc=$?
tail -2 "$OUT/prof_$TAG.log"
echo "rocprof rc=$rc"
find "$OUT/prof_$TAG" -name '*stats*' | head
exit $rc
