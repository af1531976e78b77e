#!/bin/bash
# triangular-solve tests after a tail change, then config 5 through bench.py's own leg
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_gpu_shifted.py tests/test_gpu_tri_device.py tests/test_gpu_gmres.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6/trsv_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "config5" >> gpurun_out/r6/trsv_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/extras_probe.py config5 > gpurun_out/r6/config5_default.log 2>&1
