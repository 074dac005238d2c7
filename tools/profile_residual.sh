#!/bin/bash
# Residual-kernel profiling pass (GPU box, repo root): kernel-trace stats over tools/residual_bench.py,
# then separate FETCH_SIZE / WRITE_SIZE PMC passes (one counter group per run).
# usage: tools/profile_residual.sh TAG
set -u
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rprof_$TAG" -o run -- \
    python3 "$R/tools/residual_bench.py" > "$OUT/rprof_$TAG.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/rpmcF_$TAG" -o run -- \
    python3 "$R/tools/residual_bench.py" > "$OUT/rpmcF_$TAG.log" 2>&1
rc=$?; echo "pmc FETCH_SIZE rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/rpmcW_$TAG" -o run -- \
    python3 "$R/tools/residual_bench.py" > "$OUT/rpmcW_$TAG.log" 2>&1
rc=$?; echo "pmc WRITE_SIZE rc=$rc"
exit $rc
