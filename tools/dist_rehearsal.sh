#!/bin/bash
# N > 1 rehearsal of bench.py on the one GPU of a box: bench.py --gpus N starts torch.distributed.run
# as a child and relays rank 0's line; gloo backend because RCCL refuses two ranks on one device.
# usage: tools/dist_rehearsal.sh TAG N [bench args...]
set -u
TAG=${1:-r03}
N=${2:-2}
shift 2 || true
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
GPI_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus "$N" "$@" > "$OUT/dist${N}_$TAG.json" 2> "$OUT/dist${N}_$TAG.log"
rc=$?
tail -3 "$OUT/dist${N}_$TAG.log"
cat "$OUT/dist${N}_$TAG.json"
exit $rc
