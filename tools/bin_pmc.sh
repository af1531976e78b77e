# csr_bin_kernel: timings (conditional vs unconditional level loads), then trace + PMC of uniform10m
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/bin_pmc.log
for v in "X=1" "EIGSOL_LIB_PATH=$(pwd)/build/var/lib_bincond0.so" "EIGSOL_CSR_BIN=0"; do
  echo "== $v" >> gpurun_out/bin_pmc.log
  env $v timeout -k 10 200 python3 tools/uniform_bench.py >> gpurun_out/bin_pmc.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/bin_pmc.log
bash tools/profile.sh gpurun_out/binprof uniform10m 20
for d in gpurun_out/binprof/pmc*/; do python3 tools/pmc_sum.py $d/run_counter_collection.csv csr_bin 2>&1 || true; done
