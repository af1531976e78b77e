# complex QR A/B on one box: tests of the QR module (optional), then timings over AED modes
set -o pipefail
mkdir -p gpurun_out
if [ "${ZQR_TESTS:-1}" = 1 ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_qr.py -x -v --timeout 200 --timeout-method thread > gpurun_out/zqr_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/zqr_tests.log; exit 1; }
fi
: > gpurun_out/zqr_bench.log
for n in 1024 2048 4096; do
  for cfg in "EIGSOL_ZQR_AED=0" "EIGSOL_ZQR_AED=48" "EIGSOL_ZQR_AED=64" "EIGSOL_ZQR_AED=48 EIGSOL_ZQR_AED_FULL=1"; do
    env $cfg EIGSOL_QR_STATS=1 timeout -k 10 200 python -u tools/bench_qrc.py $n >> gpurun_out/zqr_bench.log 2>&1 || exit 1
  done
done
cat gpurun_out/zqr_bench.log
tail -3 gpurun_out/zqr_tests.log
