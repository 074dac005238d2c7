#!/bin/bash
# SQ counter passes over every codec operator of the C64 step (tools/pmc_all.py, 10 launches each), one
# rocprofv3 --pmc run per counter group (<= 8 SQ counters a pass), per-operator averages via
# tools/pmc_counters_all.py.  usage: tools/r05_counters.sh TAG ["C1 C2 ..." ...]  (default groups below)
set -u
TAG=${1:-r05c}
shift || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
GROUPS=("$@")
if [ ${#GROUPS[@]} -eq 0 ]; then
    GROUPS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
            "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_INSTS_MFMA")
fi
cd /tmp && export TMPDIR=/tmp
g=0
for C in "${GROUPS[@]}"; do
    g=$((g + 1))
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/pmcS${g}_$TAG" -o run -- \
        python3 "$R/tools/pmc_all.py" "$OUT/pmc_manifest_$TAG.json" 10 > "$OUT/pmcS${g}_$TAG.log" 2>&1
    rc=$?; echo "pmc group $g rc=$rc"; [ $rc -eq 0 ] || exit $rc
    python3 "$R/tools/pmc_counters_all.py" "$OUT/pmcS${g}_$TAG" "$OUT/pmc_manifest_$TAG.json" $C \
        > "$OUT/sq${g}_$TAG.txt" 2>&1
    rc=$?; echo "counters $g rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
