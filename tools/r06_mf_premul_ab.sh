#!/bin/bash
# A/B of the premultiplied next-to-diagonal block in the large fronts' row-block solves
# (EIGSOL_MF_PREMUL, default on), 1M convection-diffusion (tools/mf_probe.py), after the
# multifrontal / GMRES / sparse-LU tests
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/mf_premul_ab.log
: > $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_multifrontal.py tests/test_gpu_gmres.py tests/test_gpu_sparse_lu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6/mf_premul_tests.log 2>&1 || exit 1
for m in 1 0 1 0; do
  echo "EIGSOL_MF_PREMUL=$m" >> $O
  EIGSOL_MF_PREMUL=$m timeout -k 10 200 python -u tools/mf_probe.py 1000 >> $O 2>&1 || exit 1
done
cat $O
