#!/bin/bash
# A/B of the shift QR's split tolerance (EIGSOL_QR_SHIFT_TOL) on config 2 (4096^2, the bench seed):
# seconds, sweeps and the LAPACK-fixture match of every setting.  Run from the repo root on the GPU box.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/shift_tol.log
for tol in 2.220446049250313e-16 1e-10 1e-8 1e-6 2.220446049250313e-16; do
  EIGSOL_QR_SHIFT_TOL=$tol timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/shift_tol.log 2>&1 || exit 1
done
