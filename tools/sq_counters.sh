#!/bin/bash
# SQ counter passes (4 counters a pass, one rocprofv3 run each) over one command; per-dispatch averages of
# every kernel whose name matches the regex, grouped by kernel name.
# usage: tools/sq_counters.sh TAG KERNEL_REGEX -- python3 tools/xxx.py args
#   SQ_PASSES: which of the passes below to run (default "1 2 3 4 5"; 6: instruction cache)
set -u
TAG=$1; KS=$2; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
g=0
P=" ${SQ_PASSES:-1 2 3 4 5} "
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
         "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_LDS" \
         "SQ_WAVES SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; do
    g=$((g + 1))
    case "$P" in *" $g "*) ;; *) continue ;; esac
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$OUT/sq_${TAG}_$g" -o run -- "$@" > "$OUT/sq_${TAG}_$g.log" 2>&1
    rc=$?; echo "pass $g rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$OUT" "$TAG" "$KS" <<'PY'
import csv, glob, re, sys
from collections import defaultdict
out, tag, ks = sys.argv[1:4]
tot = defaultdict(float); cnt = defaultdict(set)
for f in glob.glob('%s/sq_%s_*/**/*counter_collection.csv' % (out, tag), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name']
        if re.search(ks, name):
            name = re.sub(r'^(void )?(\(anonymous namespace\)::)?', '', name).split('(')[0]
            tot[(name, r['Counter_Name'])] += float(r['Counter_Value'])
            cnt[(name, r['Counter_Name'])].add(r['Dispatch_Id'])
with open('%s/sq_%s.txt' % (out, tag), 'w') as fh:
    for k in sorted(tot):
        line = '%-44s %-30s %16.1f per dispatch (%d dispatches)' % (k[0][:44], k[1], tot[k] / max(1, len(cnt[k])),
                                                                    len(cnt[k]))
        print(line); fh.write(line + '\n')
PY
