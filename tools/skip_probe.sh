#!/bin/bash
# Timing ceiling of the backward phases (timing build): per-operator profile with the weight
# gradient (1), the input gradient (2), the statistic / loss atomics (4) skipped -- results invalid,
# timing experiments only.  usage: tools/skip_probe.sh [skip values ...] (default 0 1 2 4)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/skip"
KS=${*:-0 1 2 4}
for k in $KS; do
    GPI_PHASE_TIMING=1 GPI_DBG_SKIP=$k timeout -k 10 120 python "$R/tools/skip_kprof.py" "$R/gpurun_out/skip/s$k.json" \
        > "$R/gpurun_out/skip/s$k.log" 2>&1 || { tail -3 "$R/gpurun_out/skip/s$k.log"; exit 1; }
done
python3 - "$R/gpurun_out/skip" $KS <<'PY'
import json, sys
ks = [int(k) for k in sys.argv[2:]]
d = {k: {x['op']: x['ms'] * 1e3 for x in json.load(open('%s/s%d.json' % (sys.argv[1], k)))} for k in ks}
ops = sorted(d[ks[0]], key=lambda o: -d[ks[0]][o])
print('%-42s' % 'op' + ''.join('%9s' % ('skip%d' % k) for k in ks))
for o in ops:
    print('%-42s' % o + ''.join('%9.1f' % d[k][o] for k in ks))
print('%-42s' % 'sum' + ''.join('%9.1f' % sum(d[k].values()) for k in ks))
PY
