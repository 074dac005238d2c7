#!/bin/bash
# ROM kernel A/B: phase stamps for the single-lane and the wave Cholesky (timing build)
set -u
OUT=gpurun_out; mkdir -p $OUT
for v in 0 1; do
  GPI_ROM_CHOL=$v GPI_LIB_VARIANT=timing timeout -k 10 120 python tools/rom_probe.py 50 > $OUT/rom_ab_$v.txt 2>&1 || exit $?
  echo "chol_wave=$v"; tail -2 $OUT/rom_ab_$v.txt
done
