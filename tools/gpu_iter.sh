#!/bin/bash
# One GPU iteration on the box (repo root): GPU tests, smoke, interleaved A/B bench arms, the phase probe,
# a default bench line and a rocprofv3 kernel trace -- each step optional, each under its own time limit.
# Stops at the first step that ends with anything but success (an ordinary test failure included).
# usage: tools/gpu_iter.sh TAG [ARM ...]        an arm is an environment string ("-" = the defaults)
#   IT_TESTS    pytest -k selection, "all" (default) or "none"
#   IT_SMOKE    1: __graft_entry__.smoke()
#   IT_REPS     interleaved repetitions of the arm list (default 3; no arms: no A/B)
#   IT_STEPS    bench steps per A/B arm (default 400)
#   IT_PHASE    operator names for tools/phase_probe.py (timing build) or empty
#   IT_BENCH    1: the default bench line (CPU baseline + roofline) -> gpurun_out/bench_TAG.json
#   IT_PROF     1: rocprofv3 --kernel-trace --stats of a short bench run (kernel stats + step timeline);
#               IT_PROF_UNROLL steps per graph replay there (default 1)
set -u
TAG=${1:-iter}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
SEL=${IT_TESTS:-all}
if [ "$SEL" != "none" ]; then
    if [ "$SEL" = "all" ]; then K=(); else K=(-k "$SEL"); fi
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider "${K[@]}" --timeout 300 \
        --timeout-method thread > "$OUT/tests_$TAG.log" 2>&1
    rc=$?
    grep -E "passed|failed|error" "$OUT/tests_$TAG.log" | tail -2
    [ $rc -eq 0 ] || { echo "stop after pytest rc=$rc"; tail -30 "$OUT/tests_$TAG.log"; exit $rc; }
fi
if [ "${IT_SMOKE:-0}" = "1" ]; then
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
    rc=$?; tail -1 "$OUT/smoke_$TAG.log"; [ $rc -eq 0 ] || exit $rc
fi
ARMS=("$@")
if [ ${#ARMS[@]} -gt 0 ]; then
    for rep in $(seq 1 ${IT_REPS:-3}); do
        i=0
        for E in "${ARMS[@]}"; do
            i=$((i + 1))
            [ "$E" = "-" ] && E=""
            env $E timeout -k 10 200 python -u bench.py --steps ${IT_STEPS:-400} --warmup 50 --no-cpu-baseline \
                --no-roofline > "$OUT/ab_${TAG}_${rep}_$i.log" 2> "$OUT/ab_${TAG}_${rep}_$i.err"
            rc=$?
            echo "rep $rep arm $i [${E:-defaults}]: $(tail -1 "$OUT/ab_${TAG}_${rep}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null)"
            [ $rc -eq 0 ] || { echo "stop after bench rc=$rc"; tail -5 "$OUT/ab_${TAG}_${rep}_$i.err"; exit $rc; }
        done
    done
fi
if [ -n "${IT_PHASE:-}" ]; then
    timeout -k 10 300 python -u tools/phase_probe.py $IT_PHASE > "$OUT/phase_$TAG.txt" 2>&1
    rc=$?; echo "phase probe rc=$rc"; grep -E "bwd blocks|fwd blocks|cycles/phase" "$OUT/phase_$TAG.txt" | head -40
    [ $rc -eq 0 ] || exit $rc
fi
if [ "${IT_BENCH:-0}" = "1" ]; then
    timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.log"
    rc=$?; tail -1 "$OUT/bench_$TAG.json"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${IT_PROF:-0}" = "1" ]; then
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run -- \
        python3 "$R/bench.py" --steps 20 --warmup 5 --unroll ${IT_PROF_UNROLL:-1} --no-cpu-baseline --no-roofline > "$OUT/prof_$TAG.log" 2>&1
    rc=$?
    echo "rocprof rc=$rc"
    cd "$R"
    [ $rc -eq 0 ] || exit $rc
    python3 tools/prof_summary.py "$OUT/prof_$TAG" > "$OUT/kstats_$TAG.txt" 2>&1
    python3 tools/step_timeline.py "$OUT/prof_$TAG" > "$OUT/timeline_$TAG.txt" 2>&1
    tail -3 "$OUT/timeline_$TAG.txt"
fi
exit 0
