set -u
# r05t: the delayed-side-stream epilogue test with the capped epilogue grid (default) and with the cap lifted
# (nocap build: expected to time out its flag wait and fail), then the whole handoff file on the default
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_handoff.py -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/r05t_default.log 2>&1
rc=$?; tail -6 $OUT/r05t_default.log; [ $rc -eq 0 ] || exit $rc
GPI_LIB_VARIANT=nocap timeout -k 10 300 python -u -m pytest tests/test_gpu_handoff.py -v -p no:cacheprovider -k "delayed or room" -s --timeout 200 --timeout-method thread > $OUT/r05t_nocap.log 2>&1
rc=$?; tail -6 $OUT/r05t_nocap.log; echo "nocap rc=$rc"
exit 0
