#!/bin/bash
# Complex QR grid after the round-4 AED change: AED window x nibble at 4096^2 and 1024^2 (zgeev fixtures).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/zqr_grid.log
for n in 4096 1024; do
  for aed in 40 48 56 64; do
    for nib in 14 25; do
      EIGSOL_ZQR_AED=$aed EIGSOL_ZQR_NIBBLE=$nib timeout -k 10 120 python -u tools/bench_qrc.py $n >> gpurun_out/zqr_grid.log 2>&1 || exit 1
    done
  done
done
