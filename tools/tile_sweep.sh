#!/bin/bash
# Tile-size sweep (tuning): bench + per-operator profile for each GPI_TILE_* setting.
# usage: tools/tile_sweep.sh "FWD BWD S2" ...
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/sweep"
for cfg in "$@"; do
    set -- $cfg
    tag="f$1_b$2_s$3"
    GPI_TILE_FWD=$1 GPI_TILE_BWD=$2 GPI_TILE_S2=$3 timeout -k 10 120 python "$R/bench.py" --steps 50 --warmup 10 \
        --no-cpu-baseline --kprof "$R/gpurun_out/sweep/$tag.json" > "$R/gpurun_out/sweep/$tag.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; tail -3 "$R/gpurun_out/sweep/$tag.log"; exit $rc; fi
    python3 - "$R/gpurun_out/sweep/$tag.json" "$R/gpurun_out/sweep/$tag.log" "$tag" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
line = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
f = sum(x['ms'] for x in d if x['op'].endswith('fwd')) * 1e3
b = sum(x['ms'] for x in d if x['op'].endswith('bwd')) * 1e3
print('%-18s value %9.0f  ms/step %.4f  conv fwd %6.1f us  bwd %6.1f us' % (sys.argv[3], line['value'], line['ms_per_step'], f, b))
PY
done
