set -u
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05s}
bash tools/r05_residual_pmc.sh $T
rc=$?; [ $rc -eq 0 ] || exit $rc
cp $OUT/${T}_residual_traffic.json $R/profiles/${T}_residual_traffic.json
timeout -k 10 200 python -u tools/residual_bench.py $OUT/${T}_residual_bench.json > $OUT/${T}_residual_bench.log 2>&1
rc=$?; echo "residual bench rc=$rc"; cut -c1-200 $OUT/${T}_residual_bench.log; [ $rc -eq 0 ] || exit $rc
bash tools/r05_sq.sh ${T}_band cgr_band -- python3 $R/tools/cgr_probe.py 64 4096 0 20
