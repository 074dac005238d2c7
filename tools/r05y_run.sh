set -u
# r05y: SQ counters of the fused output conv (LastTransUp.conv3, gpi_conv_loss_fused) alone, and its phase probe
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05y}
timeout -k 10 120 python3 tools/kprobe.py LastTransUp.conv3 bwd 20 > $OUT/${T}_kprobe.log 2>&1
rc=$?; tail -2 $OUT/${T}_kprobe.log; [ $rc -eq 0 ] || exit $rc
bash tools/r05_sq.sh ${T}_fused "conv_bwd_kernel<5, 1, 0, true" -- python3 $R/tools/kprobe.py LastTransUp.conv3 bwd 20 || exit 1
cd $R
GPI_PHASE_TIMING=1 timeout -k 10 200 python3 tools/phase_probe.py LastTransUp.conv3 LastTransUp.conv1 > $OUT/${T}_phase.txt 2>&1
rc=$?; cat $OUT/${T}_phase.txt | head -30; exit $rc
