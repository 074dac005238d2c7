#!/bin/bash
# Timing experiment: per-operator profile with and without the end-of-kernel fp64 atomics
# (GPI_DBG_SKIP=4; results invalid).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/atom"
for k in 0 4; do
    GPI_LIB_VARIANT=timing GPI_DBG_SKIP=$k timeout -k 10 120 python "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline \
        --kprof "$R/gpurun_out/atom/s$k.json" > "$R/gpurun_out/atom/s$k.log" 2>&1 || { tail -3 "$R/gpurun_out/atom/s$k.log"; exit 1; }
done
python3 - "$R/gpurun_out/atom" <<'PY'
import json, sys
d = {k: {x['op']: x['ms'] * 1e3 for x in json.load(open('%s/s%d.json' % (sys.argv[1], k)))} for k in (0, 4)}
ops = sorted(d[0], key=lambda o: -d[0][o])
for o in ops[:20]:
    print('%-42s %7.1f %7.1f' % (o, d[0][o], d[4][o]))
for sfx in ('fwd', 'bwd'):
    print(sfx, '%.1f %.1f' % tuple(sum(v for k, v in d[j].items() if k.endswith(sfx)) for j in (0, 4)))
PY
