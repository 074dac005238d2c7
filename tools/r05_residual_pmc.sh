#!/bin/bash
# Residual kernel: kernel-trace stats + separate FETCH_SIZE / WRITE_SIZE PMC passes over tools/residual_bench.py
# (--no-cpu), reduced to per-configuration HBM traffic (tools/residual_traffic.py, sha of stencil.hip + common.h).
# usage: tools/r05_residual_pmc.sh TAG
set -u
TAG=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/rprof_$TAG" -o run -- \
    python3 "$R/tools/residual_bench.py" --no-cpu > "$OUT/rprof_$TAG.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/rpmcF_$TAG" -o run -- \
    python3 "$R/tools/residual_bench.py" --no-cpu > "$OUT/rpmcF_$TAG.log" 2>&1
rc=$?; echo "pmc FETCH_SIZE rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/rpmcW_$TAG" -o run -- \
    python3 "$R/tools/residual_bench.py" --no-cpu > "$OUT/rpmcW_$TAG.log" 2>&1
rc=$?; echo "pmc WRITE_SIZE rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$R"
python3 tools/residual_traffic.py "$OUT/rpmcF_$TAG" "$OUT/rpmcW_$TAG" "$OUT/${TAG}_residual_traffic.json"
