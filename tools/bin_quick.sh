# csr_bin_kernel quick check: binned tests + uniform timings
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_power.py -x -q --timeout 200 --timeout-method thread -k "column_b or uniform" > gpurun_out/bin_tests.log 2>&1 || { tail -30 gpurun_out/bin_tests.log; exit 1; }
tail -1 gpurun_out/bin_tests.log
for v in "X=1" "$@"; do echo "== $v"; env $v timeout -k 10 200 python3 tools/uniform_bench.py 2>&1 | grep -v amdgpu.ids || exit 1; done
