#!/bin/bash
# Complex QR: bulges per sweep (EIGSOL_ZQR_NB; the shifts' one-wave QR runs on a 2 nb block) x AED
# full Schur (its undeflated eigenvalues as shifts, no separate shift QR) at 4096^2 / 1024^2.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/zqr_nb.log
for n in 4096 1024; do
  for nb in 12 16 24 32; do
    EIGSOL_ZQR_NB=$nb EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qrc.py $n >> gpurun_out/zqr_nb.log 2>&1 || exit 1
  done
  for aed in 48 64; do
    EIGSOL_ZQR_AED_FULL=1 EIGSOL_ZQR_AED=$aed EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qrc.py $n >> gpurun_out/zqr_nb.log 2>&1 || exit 1
  done
done
