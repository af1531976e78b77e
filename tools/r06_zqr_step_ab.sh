#!/bin/bash
# A/B of the complex one-wave QR step (EIGSOL_ZQR_STEP: 1 loads ahead + scaled reflector, 0 the round-5
# step): complex 4096^2 and 1024^2 timings against the zgeev fixtures, then the QR tests
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/zqr_step_ab.log
: > $O
for m in 0 1 0 1; do
  EIGSOL_ZQR_STEP=$m EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qrc.py 4096 >> $O 2>&1 || exit 1
done
for m in 0 1; do
  EIGSOL_ZQR_STEP=$m timeout -k 10 120 python -u tools/bench_qrc.py 1024 >> $O 2>&1 || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_qr.py tests/test_gpu_qr_stress.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6/zqr_step_tests.log 2>&1
