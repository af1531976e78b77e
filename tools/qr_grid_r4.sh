#!/bin/bash
# QR tuning grids with the round-4 exceptional-shift trigger (EXC_LEGACY=0): real 4096^2 AED window x
# bulges (bench seed: fixture match; seed 42: timing); complex 4096^2 / 1024^2 AED window x nibble.
# Run from the repo root on the GPU box.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/qr_grid.log
for seed in 20251226 42; do
  for aed in 64 80 96; do
    for nb in 28 36; do
      QR_SEED=$seed EIGSOL_QR_EXC_LEGACY=0 EIGSOL_QR_AED=$aed EIGSOL_QR_NB=$nb timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/qr_grid.log 2>&1 || exit 1
    done
  done
done
for n in 4096 1024; do
  for aed in 48 64; do
    for nib in 14 25; do
      EIGSOL_ZQR_EXC_LEGACY=0 EIGSOL_ZQR_AED=$aed EIGSOL_ZQR_NIBBLE=$nib timeout -k 10 120 python -u tools/bench_qrc.py $n >> gpurun_out/qr_grid.log 2>&1 || exit 1
    done
  done
done
