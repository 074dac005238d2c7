set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05m}
OPS="EncBlock3.denselayer1.conv1 TransDown3.conv1 TransDown3.conv2 features.conv0 DecBlock1.denselayer1.conv1 TransUp1.conv1 EncBlock2.denselayer1.conv1 TransDown2.conv2"
timeout -k 10 200 python -u tools/phase_probe.py $OPS > $OUT/${T}_phase_small.txt 2>&1
rc=$?; echo "rc=$rc"; grep -E "bwd blocks|cycles/phase|phase-1" $OUT/${T}_phase_small.txt
