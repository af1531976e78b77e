#!/bin/bash
# Hessenberg panel with two grid barriers per column (EIGSOL_HESS_MERGE=1) against three: QR 4096^2 real
# (tools/bench_qr.py) and complex (tools/bench_qrc.py), then the QR / Hessenberg tests on the merged panel
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/hess_merge_ab.log
: > $O
for m in 1 0 1 0; do
  EIGSOL_HESS_MERGE=$m timeout -k 10 120 python -u tools/bench_qr.py 4096 >> $O 2>&1 || exit 1
done
for m in 1 0; do
  EIGSOL_HESS_MERGE=$m timeout -k 10 120 python -u tools/bench_qrc.py 4096 >> $O 2>&1 || exit 1
done
EIGSOL_HESS_MERGE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_qr.py tests/test_gpu_qr_stress.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6/hess_merge_tests.log 2>&1
