# csr_bin_kernel timing probes (10M uniform, 2 MB x blocks) and its kernel trace + PMC passes
set -o pipefail
mkdir -p gpurun_out
export EIGSOL_CSR_BIN_BYTES=2097152
: > gpurun_out/bin_probe.log
for v in "" 1 2 3; do
  echo "== probe '$v'" >> gpurun_out/bin_probe.log
  if [ -n "$v" ]; then L="EIGSOL_LIB_PATH=$(pwd)/build/var/lib_binprobe$v.so"; else L="X=1"; fi
  env $L ONLY=10000000 timeout -k 10 200 python3 tools/uniform_bench.py >> gpurun_out/bin_probe.log 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/bin_probe.log
bash tools/profile.sh gpurun_out/binprof uniform10m 20
python3 tools/pmc_sum.py gpurun_out/binprof 2>&1 | tail -30
