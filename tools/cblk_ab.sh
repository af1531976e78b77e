# column-blocked uniform gathers: tests, then config 3 / uniform10m timings over block sizes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_power.py -x -v --timeout 200 --timeout-method thread -k "column_blocked or uniform" > gpurun_out/cblk_tests.log 2>&1 || { tail -30 gpurun_out/cblk_tests.log; exit 1; }
tail -3 gpurun_out/cblk_tests.log
: > gpurun_out/cblk_ab.log
for cfg in "EIGSOL_CSR_CBLK=0" "EIGSOL_CSR_CBLK_BYTES=4194304" "EIGSOL_CSR_CBLK_BYTES=3145728" "EIGSOL_CSR_CBLK_BYTES=2097152" "EIGSOL_CSR_CBLK_BYTES=1048576" "EIGSOL_CSR_CBLK_BYTES=524288"; do
  echo "== $cfg" >> gpurun_out/cblk_ab.log
  env $cfg timeout -k 10 200 python3 tools/uniform_bench.py >> gpurun_out/cblk_ab.log 2>&1 || exit 1
done
cat gpurun_out/cblk_ab.log | grep -v amdgpu.ids
