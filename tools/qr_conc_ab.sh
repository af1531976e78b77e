set -o pipefail
mkdir -p gpurun_out/r5
for m in 0 1 2 0 1 2; do
  EIGSOL_QR_CONC=$m EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/r5/qrconc.log 2>&1 || exit 1
done
for m in 0 1 2; do
  QR_SEED=7 EIGSOL_QR_CONC=$m EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qr.py 4096 >> gpurun_out/r5/qrconc.log 2>&1 || exit 1
done
