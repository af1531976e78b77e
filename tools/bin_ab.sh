# column-binned uniform gathers: tests, then config 3 / uniform10m timings over x-block sizes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_power.py -x -v --timeout 200 --timeout-method thread -k "column_b or uniform" > gpurun_out/bin_tests.log 2>&1 || { tail -30 gpurun_out/bin_tests.log; exit 1; }
tail -3 gpurun_out/bin_tests.log
: > gpurun_out/bin_ab.log
for cfg in "EIGSOL_CSR_BIN=0" "X=1" "EIGSOL_CSR_BIN_NT=512" "EIGSOL_CSR_BIN_NT=256" "EIGSOL_CSR_BIN_BYTES=1048576" "EIGSOL_CSR_BIN_BYTES=4194304" "EIGSOL_CSR_BIN_NT=512 EIGSOL_CSR_BIN_BYTES=4194304" "EIGSOL_CSR_BIN_LDS=64" "EIGSOL_CSR_BIN_LDS=64 EIGSOL_CSR_BIN_NT=512"; do
  echo "== $cfg" >> gpurun_out/bin_ab.log
  env $cfg timeout -k 10 200 python3 tools/uniform_bench.py >> gpurun_out/bin_ab.log 2>&1 || exit 1
done
cat gpurun_out/bin_ab.log | grep -v amdgpu.ids
