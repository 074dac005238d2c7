set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05e}
bash tools/r05_sq.sh ${T}_cgr cgr_stream -- python3 $R/tools/cgr_probe.py 64 4096 0 20
rc=$?; [ $rc -eq 0 ] || exit $rc
bash tools/r05_sq.sh ${T}_eb1 conv_bwd -- python3 $R/tools/kprobe.py EncBlock1.denselayer1.conv1 bwd 30
rc=$?; [ $rc -eq 0 ] || exit $rc
cd $R
ITER_TESTS=none ITER_REPS=2 ITER_STEPS=400 ITER_PROF=0 bash tools/r04_iter.sh ${T}_ab - GPI_LIB_VARIANT=w5 GPI_LIB_VARIANT=pre5
