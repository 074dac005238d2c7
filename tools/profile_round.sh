#!/bin/bash
# Profiling pass for one round (run on the GPU box, from the repo root):
#   1. rocprofv3 --kernel-trace --stats over a bench run       -> gpurun_out/prof_TAG
#   2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE) over the
#      single-operator probe of the LastTransUp convolutions    -> gpurun_out/pmc{F,W}_TAG
# Every GPU step has its own time limit and the script stops at the first failure.
# usage: tools/profile_round.sh TAG [OP_SUBSTRING]
set -u
TAG=${1:-r01}
OP=${2:-LastTransUp.conv}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcF_$TAG" -o run -- \
    python3 "$R/tools/kprobe.py" "$OP" bwd 20 > "$OUT/pmcF_$TAG.log" 2>&1
rc=$?; echo "pmc FETCH_SIZE rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcW_$TAG" -o run -- \
    python3 "$R/tools/kprobe.py" "$OP" bwd 20 > "$OUT/pmcW_$TAG.log" 2>&1
rc=$?; echo "pmc WRITE_SIZE rc=$rc"
exit $rc
