#!/bin/bash
# Round record at HEAD (GPU box, repo root): smoke, the default bench line (with the CPU baseline),
# then tools/pmc_round.sh (kernel-trace stats, FETCH_SIZE / WRITE_SIZE passes over every codec launch,
# residual stats).  Stops at the first failing step.   usage: tools/r03_final.sh TAG
set -u
TAG=${1:-r03z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke_$TAG.log" 2>&1
rc=$?; tail -2 "$OUT/smoke_$TAG.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$OUT/bench_$TAG.json" 2> "$OUT/bench_$TAG.log"
rc=$?; tail -1 "$OUT/bench_$TAG.json"; [ $rc -eq 0 ] || exit $rc
bash tools/pmc_round.sh "$TAG"
