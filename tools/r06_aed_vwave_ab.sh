#!/bin/bash
# Real AED with the Schur-vector updates on a helper wave (EIGSOL_QR_AED_VWAVE=1, default) against one wave (0):
# (the helper-wave AED, EIGSOL_QR_AED_VWAVE, was measured slower and removed; the script documents profiles/r06_aed_vwave_ab.log)
# the bitwise test, then QR 4096^2 (tools/bench_qr.py) alternating, then the QR tests
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/aed_vwave_ab.log
: > $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_qr.py -x -q --timeout 200 --timeout-method thread -k "aed_v_helper" > gpurun_out/r6/aed_vwave_tests.log 2>&1 || exit 1
for v in 1 0 1 0; do
  EIGSOL_QR_AED_VWAVE=$v timeout -k 10 120 python3 -u tools/bench_qr.py 4096 >> $O 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_qr.py tests/test_gpu_qr_stress.py -x -q --timeout 200 --timeout-method thread >> gpurun_out/r6/aed_vwave_tests.log 2>&1
