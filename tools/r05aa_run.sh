set -u
# r05aa: VALU / SALU / LDS instruction attribution of the fused output conv by the timing build's work-skip
# switches (GPI_DBG_SKIP: 0 all, 1 no weight gradient, 2 no input gradient, 8 return after the operand loads),
# one 8-counter SQ pass each over tools/kprobe.py (the launch alone)
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05aa}
cd /tmp && export TMPDIR=/tmp
for m in 0 1 2 8; do
  GPI_PHASE_TIMING=1 GPI_DBG_SKIP=$m timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS \
    --output-format csv -d "$OUT/${T}_skip$m" -o run -- python3 $R/tools/kprobe.py LastTransUp.conv3 bwd 20 > "$OUT/${T}_skip$m.log" 2>&1
  rc=$?; echo "skip $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" "$T" <<'PY'
import csv, glob, sys
from collections import defaultdict
out, tag = sys.argv[1:3]
for m in (0, 1, 2, 8):
    tot = defaultdict(float); cnt = defaultdict(set)
    for f in glob.glob('%s/%s_skip%d/**/*counter_collection.csv' % (out, tag, m), recursive=True):
        for r in csv.DictReader(open(f)):
            if 'conv_bwd_kernel<5, 1, 0, true' in r['Kernel_Name']:
                tot[r['Counter_Name']] += float(r['Counter_Value']); cnt[r['Counter_Name']].add(r['Dispatch_Id'])
    w = tot['SQ_WAVES'] / max(1, len(cnt['SQ_WAVES']))
    per = {k: tot[k] / max(1, len(cnt[k])) / max(w, 1) for k in tot}
    print('skip %d: waves %d  per wave: ' % (m, w) + '  '.join('%s %.0f' % (k.replace('SQ_', ''), v) for k, v in sorted(per.items()) if k != 'SQ_WAVES'))
PY
