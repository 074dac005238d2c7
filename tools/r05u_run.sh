set -u
# r05u: multigrid-preconditioned FOM solve: FOM tests, then the FOM bench with the multigrid from 128^2
# (default) and forced from 32^2, and the Jacobi form everywhere (GPI_FOM_MG_MIN=0)
R=$(pwd); OUT=$R/gpurun_out; mkdir -p $OUT
T=${1:-r05u}
timeout -k 10 400 python -u -m pytest tests/test_gpu_fom.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/${T}_tests.log 2>&1
rc=$?; tail -4 $OUT/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
for arm in 128 32 0; do
  GPI_FOM_MG_MIN=$arm timeout -k 10 300 python -u tools/fom_bench.py --grids 32,64,128,256 --no-cpu --out $OUT/${T}_fom_$arm.json > $OUT/${T}_fom_$arm.log 2>&1
  rc=$?; echo "arm MG_MIN=$arm rc=$rc"; python3 -c "
import json,sys
for l in open('$OUT/${T}_fom_$arm.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['metric'], round(d['value']), 'iters', d['iters_mean'], d['iters_max'], 'ms', round(d['ms'],2))"
  [ $rc -eq 0 ] || exit $rc
done
