#!/bin/bash
# Multifrontal set-up with the latency-restructured inverse forms (mf_invform2_kernel, default) against round 5's
# kernel (EIGSOL_MF_INVFORM=1): 1M convection-diffusion factor seconds and ms per iteration (tools/mf_probe.py),
# the inverse-form tests first
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/mf_invform_ab.log
: > $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multifrontal.py -x -q --timeout 200 --timeout-method thread -k "inverse_forms" > gpurun_out/r6/mf_invform_tests.log 2>&1 || exit 1
for m in 2 1 2 1; do
  echo "EIGSOL_MF_INVFORM=$m" >> $O
  EIGSOL_MF_INVFORM=$m EIGSOL_MF_DEBUG=1 timeout -k 10 200 python -u tools/mf_probe.py 1000 >> $O 2>&1 || exit 1
done
