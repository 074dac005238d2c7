#!/bin/bash
# Per-kernel A/B under rocprofv3 --kernel-trace --stats: one short bench run per environment string,
# then the rows of the stats summary whose kernel name matches PATTERN.  Each run has its own limit
# and a failure ends the script.
# usage: tools/kstat_ab.sh TAG PATTERN "ENV1" "ENV2" ...   (an environment string "-" = defaults)
set -u
TAG=${1:-kab}
PAT=${2:-head}
shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for E in "$@"; do
    i=$((i + 1))
    [ "$E" = "-" ] && E=""
    for kv in $E; do export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kab_${TAG}_$i" -o run -- \
        python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu-baseline --no-roofline \
        > "$OUT/kab_${TAG}_$i.log" 2>&1
    rc=$?
    for kv in $E; do unset "${kv%%=*}"; done
    echo "[$i] ${E:-defaults} rc=$rc $(tail -1 "$OUT/kab_${TAG}_$i.log" | cut -c1-160)"
    [ $rc -eq 0 ] || exit $rc
    f=$(ls "$OUT/kab_${TAG}_$i"/*/run_kernel_stats.csv "$OUT/kab_${TAG}_$i"/run_kernel_stats.csv 2>/dev/null | head -1)
    python3 - "$f" "$PAT" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if sys.argv[2] in r['Name']:
        print('   %-60s calls %6s avg %8.2f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs']) / 1e3))
EOF
done
