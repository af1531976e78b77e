#!/bin/bash
# Real QR grid after the exceptional-shift fix: bulges per sweep (EIGSOL_QR_NB, up to 48) x AED window,
# two seeds (bench seed: fixture match).  Run from the repo root on the GPU box.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/qr_grid_b.log
for seed in 20251226 42; do
  for aed in 56 64; do
    for nb in 32 40 48; do
      QR_SEED=$seed EIGSOL_QR_AED=$aed EIGSOL_QR_NB=$nb timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/qr_grid_b.log 2>&1 || exit 1
    done
  done
done
