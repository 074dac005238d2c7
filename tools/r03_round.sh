#!/bin/bash
# One GPU pass: the whole GPU test suite, then bench A/B arms (tools/ab_env.sh, AB_SKIP_TESTS).
# usage: tools/r03_round.sh TAG "ENV1" "ENV2" ...   (stops at the first failing step)
set -u
TAG=${1:-r03}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$OUT/t_$TAG.log" 2>&1
rc=$?; tail -3 "$OUT/t_$TAG.log"; [ $rc -eq 0 ] || exit $rc
[ $# -gt 0 ] || exit 0
AB_SKIP_TESTS=1 AB_STEPS=${AB_STEPS:-600} bash tools/ab_env.sh "$TAG" "$@"
rc=$?; [ $rc -eq 0 ] || exit $rc
if [ -n "${NB_AB:-}" ]; then
    for E in GPI_PE_SHARED_GRADS=1 GPI_PE_SHARED_GRADS=0 GPI_PE_SHARED_GRADS=1 GPI_PE_SHARED_GRADS=0; do
        env $E timeout -k 10 200 python -u tools/notebook_bench.py 2000 > "$OUT/nb_${TAG}_$E.log" 2>&1 || exit $?
        echo "$E: $(tail -1 "$OUT/nb_${TAG}_$E.log")"
    done
fi
