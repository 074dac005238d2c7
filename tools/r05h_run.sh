set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05h}
OPS="EncBlock1.denselayer1.conv1 DecBlock3.denselayer1.conv1 LastTransUp.conv1"
for arm in "-" "GPI_LIB_VARIANT=novdg3" "GPI_DBG_SKIP=2"; do
  E=""; [ "$arm" = "-" ] || E="$arm"
  env $E GPI_PROBE_HALVES=1 timeout -k 10 200 python -u tools/phase_probe.py $OPS > $OUT/${T}_phase_$(echo $arm | tr = _).txt 2>&1
  rc=$?; echo "== [$arm] rc=$rc"; grep -E "bwd blocks|cycles/phase|half" $OUT/${T}_phase_$(echo $arm | tr = _).txt; [ $rc -eq 0 ] || exit $rc
done
