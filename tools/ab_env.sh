#!/bin/bash
# A/B of tuning environments on the GPU box: codec parity tests once, then one bench run (with the
# per-operator profile) per environment string.  Every run has its own time limit; a crash ends the
# script.  usage: tools/ab_env.sh TAG "ENV1" "ENV2" ...   (an environment string "-" = defaults)
set -u
TAG=${1:-ab}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
if [ -z "${AB_SKIP_TESTS:-}" ]; then
    timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c64.py \
        -k "${AB_TESTS:-codec or elbo or fused or dropout or c64}" -q -p no:cacheprovider \
        --timeout 300 --timeout-method thread > "$OUT/ab_tests_$TAG.log" 2>&1
    rc=$?
    tail -2 "$OUT/ab_tests_$TAG.log"
    if [ $rc -ne 0 ]; then echo "stop after pytest rc=$rc"; exit $rc; fi
fi
i=0
for E in "$@"; do
    i=$((i + 1))
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 200 python -u bench.py --steps ${AB_STEPS:-300} --warmup 30 --no-cpu-baseline \
        --kprof "$OUT/kprof_${TAG}_$i.json" > "$OUT/bench_${TAG}_$i.log" 2> "$OUT/bench_${TAG}_$i.err"
    rc=$?
    echo "[$i] ${E:-defaults}: $(tail -1 "$OUT/bench_${TAG}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])' 2>/dev/null)"
    if [ $rc -ne 0 ]; then echo "stop after bench rc=$rc"; tail -5 "$OUT/bench_${TAG}_$i.err"; exit $rc; fi
done
