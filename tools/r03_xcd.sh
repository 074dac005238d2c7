#!/bin/bash
# XCD-aware tile order (GPI_XCD_TILES): codec parity tests with the default (on), bench A/B
# interleaved off/on/off/on, then the two PMC traffic passes of every codec launch with the default.
# Every GPU step has its own limit; the script stops at the first failure.
# usage: tools/r03_xcd.sh TAG
set -u
TAG=${1:-r03x}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c64.py -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > "$OUT/t_$TAG.log" 2>&1
rc=$?; tail -2 "$OUT/t_$TAG.log"; [ $rc -eq 0 ] || exit $rc
i=0
for E in GPI_XCD_TILES=0 GPI_XCD_TILES=1 GPI_XCD_TILES=0 GPI_XCD_TILES=1; do
    i=$((i + 1))
    env $E timeout -k 10 200 python -u bench.py --steps 600 --warmup 100 --no-cpu-baseline \
        --kprof "$OUT/kprof_${TAG}_$i.json" > "$OUT/bench_${TAG}_$i.log" 2> "$OUT/bench_${TAG}_$i.err"
    rc=$?
    echo "[$i] $E: $(tail -1 "$OUT/bench_${TAG}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"])' 2>/dev/null)"
    [ $rc -eq 0 ] || { tail -5 "$OUT/bench_${TAG}_$i.err"; exit $rc; }
done
for V in full no_side full no_side; do
    timeout -k 10 120 python tools/critpath_probe.py $V 600 >> "$OUT/crit_$TAG.txt" 2>&1 || exit $?
done
cat "$OUT/crit_$TAG.txt"
for E in - DEBUG_HIP_FORCE_GRAPH_QUEUES=1 GPI_GRAPH_MODE=segments; do
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 120 python tools/host_walk_probe.py 200 >> "$OUT/hostwalk_$TAG.txt" 2>&1 || exit $?
done
cat "$OUT/hostwalk_$TAG.txt"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmc${C:0:1}_$TAG" -o run -- \
        python3 "$R/tools/pmc_all.py" "$OUT/pmc_manifest_$TAG.json" 10 > "$OUT/pmc${C:0:1}_$TAG.log" 2>&1
    rc=$?; echo "pmc $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 "$R/tools/pmc_traffic_all.py" "$OUT/pmcF_$TAG" "$OUT/pmcW_$TAG" "$OUT/pmc_manifest_$TAG.json" \
    "$OUT/traffic_$TAG.json" > "$OUT/traffic_$TAG.txt" 2>&1
rc=$?; echo "traffic rc=$rc"; grep -E "LastTransUp|total" "$OUT/traffic_$TAG.txt"
exit $rc
