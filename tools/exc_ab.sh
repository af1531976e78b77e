#!/bin/bash
# A/B of the exceptional-shift trigger (round 4 fix vs round 3's legacy test that also fired right
# after an AED deflation): real QR 4096^2 (two seeds) and complex QR 4096^2 / 1024^2.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/exc_ab.log
for leg in 1 0; do
  for seed in 20251226 42; do
    QR_SEED=$seed EIGSOL_QR_EXC_LEGACY=$leg EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/exc_ab.log 2>&1 || exit 1
  done
  EIGSOL_ZQR_EXC_LEGACY=$leg EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qrc.py 4096 >> gpurun_out/exc_ab.log 2>&1 || exit 1
  EIGSOL_ZQR_EXC_LEGACY=$leg EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qrc.py 1024 >> gpurun_out/exc_ab.log 2>&1 || exit 1
done
