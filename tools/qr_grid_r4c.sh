#!/bin/bash
# Real QR after the round-4 shift changes: full-Schur AED (its undeflated eigenvalues as the shifts,
# EIGSOL_QR_AED_EARLY=0) against the early-stop default, and the nibble, two seeds.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/qr_grid_c.log
for seed in 20251226 42; do
  for aed in 64 96; do
    QR_SEED=$seed EIGSOL_QR_AED_EARLY=0 EIGSOL_QR_AED=$aed timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/qr_grid_c.log 2>&1 || exit 1
  done
  for nib in 20 30 40; do
    QR_SEED=$seed EIGSOL_QR_NIBBLE=$nib timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/qr_grid_c.log 2>&1 || exit 1
  done
done
