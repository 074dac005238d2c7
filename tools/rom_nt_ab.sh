#!/bin/bash
# ROM workgroup-width A/B (GPI_ROM_FAST_NT = 256 / 512 / 1024): ROM parity tests, then the isolated
# launch time (tools/rom_probe.py) and the phase stamps (timing build) per width.  GPU box, repo root.
set -u
OUT=gpurun_out; mkdir -p $OUT
for nt in 256 512 1024; do
  GPI_ROM_FAST_NT=$nt timeout -k 10 300 python -u -m pytest tests/test_gpu_c64.py tests/test_gpu_parity.py \
      -k "rom or fused_step" -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/rom_nt_t_$nt.log 2>&1
  rc=$?; echo "nt=$nt tests: $(tail -1 $OUT/rom_nt_t_$nt.log)"; [ $rc -eq 0 ] || exit $rc
  GPI_ROM_FAST_NT=$nt timeout -k 10 120 python tools/rom_probe.py 200 > $OUT/rom_nt_$nt.txt 2>&1 || exit $?
  GPI_ROM_FAST_NT=$nt GPI_LIB_VARIANT=timing timeout -k 10 120 python tools/rom_probe.py 50 > $OUT/rom_nt_phase_$nt.txt 2>&1 || exit $?
  tail -1 $OUT/rom_nt_$nt.txt; grep phases $OUT/rom_nt_phase_$nt.txt
done
