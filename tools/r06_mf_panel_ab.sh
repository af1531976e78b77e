#!/bin/bash
# Multifrontal numeric factorization with mf_panel2_kernel (default) against round 5's panel kernel (EIGSOL_MF_PANEL=1):
# (the EIGSOL_MF_PANEL switch was removed with the kernel; the script documents profiles/r06_mf_panel_ab.log)
# the panel / static-pivot / bitwise tests, then 1M convection-diffusion set-up laps (tools/mf_probe.py, EIGSOL_MF_DEBUG=1)
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/mf_panel_ab.log
: > $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multifrontal.py -x -q --timeout 200 --timeout-method thread -k "panel2 or pivot or fixture" > gpurun_out/r6/mf_panel_tests.log 2>&1 || exit 1
for m in 2 1 2 1; do
  echo "EIGSOL_MF_PANEL=$m" >> $O
  EIGSOL_MF_PANEL=$m EIGSOL_MF_DEBUG=1 timeout -k 10 200 python -u tools/mf_probe.py 1000 >> $O 2>&1 || exit 1
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_multifrontal.py tests/test_gpu_gmres.py -x -q --timeout 200 --timeout-method thread >> gpurun_out/r6/mf_panel_tests.log 2>&1
