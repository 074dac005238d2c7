set -u
# r05ac: instruction attribution by phase (timing build's work-skip switches) of the two largest 3x3 stride-1
# backwards, LastTransUp.conv1 and EncBlock1.denselayer1.conv1, each alone under tools/kprobe.py
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05ac}
cd /tmp && export TMPDIR=/tmp
for op in LastTransUp.conv1 EncBlock1.denselayer1.conv1; do
for m in 0 1 2 8; do
  GPI_PHASE_TIMING=1 GPI_DBG_SKIP=$m timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS \
    --output-format csv -d "$OUT/${T}_${op}_skip$m" -o run -- python3 $R/tools/kprobe.py $op bwd 20 > "$OUT/${T}_${op}_skip$m.log" 2>&1
  rc=$?; echo "$op skip $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
done
python3 - "$OUT" "$T" <<'PY'
import csv, glob, sys
from collections import defaultdict
out, tag = sys.argv[1:3]
for op in ('LastTransUp.conv1', 'EncBlock1.denselayer1.conv1'):
    for m in (0, 1, 2, 8):
        tot = defaultdict(float); cnt = defaultdict(set)
        for f in glob.glob('%s/%s_%s_skip%d/**/*counter_collection.csv' % (out, tag, op, m), recursive=True):
            rows = [r for r in csv.DictReader(open(f)) if 'conv_bwd_kernel<3, 1, 0' in r['Kernel_Name']]
            ids = sorted({int(r['Dispatch_Id']) for r in rows})[-20:]      # the probe's 20 launches (the warm step's come first)
            for r in rows:
                if int(r['Dispatch_Id']) in ids:
                    tot[r['Counter_Name']] += float(r['Counter_Value']); cnt[r['Counter_Name']].add(r['Dispatch_Id'])
        w = tot['SQ_WAVES'] / max(1, len(cnt['SQ_WAVES']))
        per = {k: tot[k] / max(1, len(cnt[k])) / max(w, 1) for k in tot}
        print('%s skip %d: waves %d  per wave: ' % (op, m, w) + '  '.join('%s %.0f' % (k.replace('SQ_', ''), v) for k, v in sorted(per.items()) if k != 'SQ_WAVES'))
PY
