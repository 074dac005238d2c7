set -u
# r05o: one slab row per tile (GPI_LSUM) re-measured on the current kernels: all planes (1), <= 16^2 (2)
T=${1:-r05o}
ITER_TESTS=none ITER_REPS=3 ITER_STEPS=400 ITER_PROF=0 bash tools/r04_iter.sh ${T}_ab - GPI_LSUM=1 GPI_LSUM=2
