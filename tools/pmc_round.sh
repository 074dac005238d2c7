#!/bin/bash
# Profiling pass (GPU box, repo root): kernel-trace stats of a bench run, then two PMC passes
# (FETCH_SIZE, WRITE_SIZE; separate runs, counters only with --kernel-trace-free collection) over every
# codec operator, then the residual-kernel stats.  Stops at the first failing step.
# usage: tools/pmc_round.sh TAG
set -u
TAG=${1:-r02}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$TAG" -o run -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-roofline > "$OUT/prof_$TAG.log" 2>&1
rc=$?; echo "kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
find "$OUT/prof_$TAG" -type f | head -20
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcF_$TAG" -o run -- \
    python3 "$R/tools/pmc_all.py" "$OUT/pmc_manifest_$TAG.json" 10 > "$OUT/pmcF_$TAG.log" 2>&1
rc=$?; echo "pmc FETCH_SIZE rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcW_$TAG" -o run -- \
    python3 "$R/tools/pmc_all.py" "$OUT/pmc_manifest_$TAG.json" 10 > "$OUT/pmcW_$TAG.log" 2>&1
rc=$?; echo "pmc WRITE_SIZE rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 "$R/tools/pmc_traffic_all.py" "$OUT/pmcF_$TAG" "$OUT/pmcW_$TAG" "$OUT/pmc_manifest_$TAG.json" \
    "$OUT/traffic_$TAG.json" > "$OUT/traffic_$TAG.txt" 2>&1
rc=$?; echo "traffic rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/profres_$TAG" -o run -- \
    python3 "$R/tools/residual_bench.py" > "$OUT/profres_$TAG.log" 2>&1
rc=$?; echo "residual kernel-trace rc=$rc"
exit $rc
