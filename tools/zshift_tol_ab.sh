#!/bin/bash
# A/B of the complex shifts' split tolerance (EIGSOL_ZQR_SHIFT_TOL) at 4096^2 and 1024^2, both matched
# to the zgeev fixtures.  Run from the repo root on the GPU box.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/zshift_tol.log
for n in 4096 1024; do
  for tol in 2.220446049250313e-16 1e-6 1e-4 1e-3; do
    EIGSOL_ZQR_SHIFT_TOL=$tol EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qrc.py $n >> gpurun_out/zshift_tol.log 2>&1 || exit 1
  done
done
