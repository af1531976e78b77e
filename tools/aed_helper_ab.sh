#!/bin/bash
# A/B of the AED's V helper wave (EIGSOL_QR_AED_HELPER) on config 2, two seeds; the eigenvalues must
# match bitwise (max_match_dist identical for the bench seed).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/aed_helper.log
for h in 0 1 0 1; do
  for seed in 20251226 42; do
    QR_SEED=$seed EIGSOL_QR_AED_HELPER=$h EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/aed_helper.log 2>&1 || exit 1
  done
done
