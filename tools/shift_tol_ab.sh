#!/bin/bash
# A/B of the shift QR's split tolerance (EIGSOL_QR_SHIFT_TOL) on 4096^2 N(0,1) matrices (the bench
# seed, matched to the LAPACK fixture, and two more seeds, timing only): seconds and sweeps.
# Run from the repo root on the GPU box.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/shift_tol.log
for seed in 20251226 42 7; do
  for tol in 2.220446049250313e-16 1e-6 1e-5 1e-4 1e-3; do
    QR_SEED=$seed EIGSOL_QR_SHIFT_TOL=$tol timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/shift_tol.log 2>&1 || exit 1
  done
done
