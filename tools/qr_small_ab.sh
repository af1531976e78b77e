#!/bin/bash
# Real QR: order of the blocks finished by the one-wave solver (EIGSOL_QR_SMALL), two seeds.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/qr_small.log
for sm in 128 96 64 128; do
  for seed in 20251226 42; do
    QR_SEED=$seed EIGSOL_QR_SMALL=$sm timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/qr_small.log 2>&1 || exit 1
  done
done
