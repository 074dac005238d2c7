#!/bin/bash
# Interleaved A/B of bench configurations on the GPU box (repo root): for each rep, each config, each arm
# (an environment string, "-" = defaults) one short bench run -> gpurun_out/cab_TAG_*.log; prints ms/step.
# usage: tools/config_ab.sh TAG REPS "CONFIG ..." ARM [ARM ...]
set -u
TAG=$1; REPS=$2; CFGS=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
for rep in $(seq 1 $REPS); do
    for cfg in $CFGS; do
        i=0
        for E in "$@"; do
            i=$((i + 1))
            [ "$E" = "-" ] && E=""
            env $E timeout -k 10 200 python -u bench.py --config $cfg --steps ${CAB_STEPS:-100} --warmup 20 --no-cpu-baseline \
                --no-roofline > "$OUT/cab_${TAG}_${rep}_${cfg}_$i.log" 2> "$OUT/cab_${TAG}_${rep}_${cfg}_$i.err"
            rc=$?
            echo "rep $rep $cfg arm $i [${E:-defaults}]: $(tail -1 "$OUT/cab_${TAG}_${rep}_${cfg}_$i.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("conv_shapes"))' 2>/dev/null)"
            [ $rc -eq 0 ] || { echo "stop after bench rc=$rc"; tail -5 "$OUT/cab_${TAG}_${rep}_${cfg}_$i.err"; exit $rc; }
        done
    done
done
exit 0
