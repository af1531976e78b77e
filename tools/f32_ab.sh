# f32 slice pipeline variants (build/var/lib_f32*.so) on band10m / 1M band, base library first
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/f32_ab.log
echo "== base" >> gpurun_out/f32_ab.log
timeout -k 10 120 python3 tools/f32_probe.py >> gpurun_out/f32_ab.log 2>&1 || exit 1
for v in a b c d; do
  echo "== f32$v" >> gpurun_out/f32_ab.log
  EIGSOL_LIB_PATH=$PWD/build/var/lib_f32$v.so timeout -k 10 120 python3 tools/f32_probe.py >> gpurun_out/f32_ab.log 2>&1 || exit 1
done
for b in 3 4; do
  echo "== base blocks/CU $b" >> gpurun_out/f32_ab.log
  EIGSOL_CSR_BLOCKS_PER_CU=$b timeout -k 10 120 python3 tools/f32_probe.py >> gpurun_out/f32_ab.log 2>&1 || exit 1
done
cat gpurun_out/f32_ab.log
