#!/bin/bash
# One performance iteration on the GPU box: codec parity tests, then the bench with the per-operator
# profile.  usage: tools/perf_iter.sh TAG [pytest -k expression]
set -u
TAG=${1:-it}
K=${2:-"codec or elbo or fused or dropout or c64"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c64.py -k "$K" -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > "$OUT/perf_tests_$TAG.log" 2>&1
rc=$?
tail -2 "$OUT/perf_tests_$TAG.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 200 --warmup 30 --no-cpu-baseline --kprof "$OUT/kprof_$TAG.json" \
    > "$OUT/bench_$TAG.log" 2> "$OUT/bench_$TAG.err"
rc2=$?
tail -1 "$OUT/bench_$TAG.log" | cut -c1-200
exit $rc2
