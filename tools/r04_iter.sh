#!/bin/bash
# One round-4 GPU iteration: GPU tests (optional subset), interleaved A/B bench arms, rocprof kernel trace.
# Each GPU step has its own time limit; anything but a clean exit / ordinary test failure ends the script.
# usage: tools/r04_iter.sh TAG [ARM ...]   (an arm is an environment string, "-" = defaults)
#   ITER_TESTS   pytest selection (-k expression) or "none" / "all" (default all)
#   ITER_REPS    interleaved repetitions of the arm list (default 2)
#   ITER_PROF    0 to skip the rocprof pass
set -u
TAG=${1:-iter}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
SEL=${ITER_TESTS:-all}
if [ "$SEL" != "none" ]; then
    if [ "$SEL" = "all" ]; then K=(); else K=(-k "$SEL"); fi
    timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider "${K[@]}" --timeout 300 \
        --timeout-method thread > "$OUT/tests_$TAG.log" 2>&1
    rc=$?
    tail -3 "$OUT/tests_$TAG.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after pytest rc=$rc"; exit $rc; fi
fi
ARMS=("$@")
[ ${#ARMS[@]} -eq 0 ] && ARMS=("-")
for rep in $(seq 1 ${ITER_REPS:-2}); do
    i=0
    for E in "${ARMS[@]}"; do
        i=$((i + 1))
        [ "$E" = "-" ] && E=""
        env $E timeout -k 10 200 python -u bench.py --steps ${ITER_STEPS:-400} --warmup 50 --no-cpu-baseline \
            --no-roofline > "$OUT/bench_${TAG}_${rep}_$i.log" 2> "$OUT/bench_${TAG}_${rep}_$i.err"
        rc=$?
        echo "rep $rep arm $i [${E:-defaults}]: $(tail -1 "$OUT/bench_${TAG}_${rep}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null)"
        if [ $rc -ne 0 ]; then echo "stop after bench rc=$rc"; tail -5 "$OUT/bench_${TAG}_${rep}_$i.err"; exit $rc; fi
    done
done
if [ "${ITER_PROF:-1}" != "0" ]; then
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run -- \
        python3 "$R/bench.py" --steps 20 --warmup 5 --unroll 1 --no-cpu-baseline --no-roofline > "$OUT/prof_$TAG.log" 2>&1
    rc=$?
    echo "rocprof rc=$rc"
    cd "$R"
    if [ $rc -eq 0 ]; then
        python3 tools/prof_summary.py "$OUT/prof_$TAG" > "$OUT/kstats_$TAG.txt" 2>&1
        python3 tools/step_timeline.py "$OUT/prof_$TAG" > "$OUT/timeline_$TAG.txt" 2>&1
        tail -3 "$OUT/timeline_$TAG.txt"
    fi
fi
exit 0
