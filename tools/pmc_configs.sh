#!/bin/bash
# Per-operator HBM traffic (two separate PMC passes, FETCH_SIZE and WRITE_SIZE, over tools/pmc_all.py)
# for each bench configuration named on the command line -> gpurun_out/traffic_TAG_CONFIG.{json,txt}.
# Stops at the first failing step.  usage: tools/pmc_configs.sh TAG CONFIG [CONFIG ...]
set -u
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for CFG in "$@"; do
    M="$OUT/pmc_manifest_${TAG}_$CFG.json"
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmcF_${TAG}_$CFG" -o run -- \
        python3 "$R/tools/pmc_all.py" "$M" 10 "$CFG" > "$OUT/pmcF_${TAG}_$CFG.log" 2>&1
    rc=$?; echo "$CFG pmc FETCH_SIZE rc=$rc"; [ $rc -eq 0 ] || exit $rc
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmcW_${TAG}_$CFG" -o run -- \
        python3 "$R/tools/pmc_all.py" "$M" 10 "$CFG" > "$OUT/pmcW_${TAG}_$CFG.log" 2>&1
    rc=$?; echo "$CFG pmc WRITE_SIZE rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 "$R/tools/pmc_traffic_all.py" "$OUT/pmcF_${TAG}_$CFG" "$OUT/pmcW_${TAG}_$CFG" "$M" \
        "$OUT/traffic_${TAG}_$CFG.json" > "$OUT/traffic_${TAG}_$CFG.txt" 2>&1
    rc=$?; echo "$CFG traffic rc=$rc"; [ $rc -eq 0 ] || exit $rc
    # the traffic file where bench.py looks for it (TRAFFIC_FILES), then the config's CPU-baseline +
    # roofline bench line (short)
    cd "$R"
    P=${TPFX:-r05}
    if [ "$CFG" = "c64" ]; then TF=${P}_traffic.json; else TF=${P}_traffic_$CFG.json; fi
    cp "$OUT/traffic_${TAG}_$CFG.json" "$R/profiles/$TF"
    timeout -k 10 300 python3 bench.py --config "$CFG" --steps 50 --warmup 10 > "$OUT/bench_${TAG}_$CFG.json" \
        2> "$OUT/bench_${TAG}_$CFG.err"
    rc=$?; echo "$CFG bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
    cd /tmp
done
exit 0
