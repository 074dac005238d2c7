#!/bin/bash
# Timing ceiling of the backward phases: per-operator profile with the weight gradient (1), the
# input gradient (2) or both (3) skipped (results invalid; timing experiments only).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/skip"
for k in 0 1 2 3; do
    GPI_DBG_SKIP=$k timeout -k 10 120 python "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline \
        --kprof "$R/gpurun_out/skip/s$k.json" > "$R/gpurun_out/skip/s$k.log" 2>&1 || { tail -3 "$R/gpurun_out/skip/s$k.log"; exit 1; }
done
python3 - "$R/gpurun_out/skip" <<'PY'
import json, sys
d = {k: {x['op']: x['ms'] * 1e3 for x in json.load(open('%s/s%d.json' % (sys.argv[1], k)))} for k in range(4)}
ops = [o for o in d[0] if o.endswith('bwd')]
ops.sort(key=lambda o: -d[0][o])
print('%-42s %7s %7s %7s %7s' % ('op', 'full', '-wgrad', '-dgrad', '-both'))
for o in ops:
    print('%-42s %7.1f %7.1f %7.1f %7.1f' % (o, d[0][o], d[1][o], d[2][o], d[3][o]))
print('%-42s %7.1f %7.1f %7.1f %7.1f' % ('sum', *[sum(d[k][o] for o in ops) for k in range(4)]))
PY
