#!/bin/bash
# A/B of fused height launches in the multifrontal solve (EIGSOL_MF_FUSE_BIG: one forward launch per height; EIGSOL_MF_FUSE_ASM measured earlier, profiles/r06_mf_fuse_ab.log), 1M
# convection-diffusion (tools/mf_probe.py), then the multifrontal / GMRES tests
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/mf_fuse2_ab.log
: > $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multifrontal.py -x -q --timeout 200 --timeout-method thread -k "fused" > gpurun_out/r6/mf_fuse2_tests.log 2>&1 || exit 1
for m in 1 0 1 0; do
  echo "EIGSOL_MF_FUSE_BIG=$m" >> $O
  EIGSOL_MF_FUSE_BIG=$m timeout -k 10 200 python -u tools/mf_probe.py 1000 >> $O 2>&1 || exit 1
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_multifrontal.py tests/test_gpu_gmres.py -x -q --timeout 200 --timeout-method thread >> gpurun_out/r6/mf_fuse2_tests.log 2>&1
