#!/bin/bash
# Real QR tuning grid after the shift-tolerance change (round 4): AED window x bulges per sweep x
# nibble on 4096^2 (bench seed: fixture match; seed 42: timing).  Run from the repo root on the GPU box.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/qr_grid.log
for seed in 20251226 42; do
  for aed in 64 80 96; do
    for nb in 28 36; do
      for nib in 30 50; do
        QR_SEED=$seed EIGSOL_QR_AED=$aed EIGSOL_QR_NB=$nb EIGSOL_QR_NIBBLE=$nib timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/qr_grid.log 2>&1 || exit 1
      done
    done
  done
done
