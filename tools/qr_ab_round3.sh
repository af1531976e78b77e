# QR A/B (round 3): real early-stop AED grid at 4096; complex bulge count / chains at 1024
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/qr_ab3.log
for a in 48 56 64; do for nib in 30 50; do for nb in 28 36; do
  echo "real EIGSOL_QR_AED=$a NIBBLE=$nib NB=$nb" >> gpurun_out/qr_ab3.log
  EIGSOL_QR_AED_EARLY=1 EIGSOL_QR_AED=$a EIGSOL_QR_NIBBLE=$nib EIGSOL_QR_NB=$nb EIGSOL_QR_STATS=1 timeout -k 10 100 python -u tools/bench_qr.py 4096 >> gpurun_out/qr_ab3.log 2>&1 || exit 1
done; done; done
for cfg in "EIGSOL_ZQR_AED=48" "EIGSOL_ZQR_AED=48 EIGSOL_ZQR_NB=24 EIGSOL_ZQR_GROUPS=3" "EIGSOL_ZQR_AED=48 EIGSOL_ZQR_NB=32 EIGSOL_ZQR_GROUPS=4" "EIGSOL_ZQR_AED=64 EIGSOL_ZQR_NB=32 EIGSOL_ZQR_GROUPS=4" "EIGSOL_ZQR_AED=32 EIGSOL_ZQR_NB=32 EIGSOL_ZQR_GROUPS=4"; do
  env $cfg EIGSOL_QR_STATS=1 timeout -k 10 100 python -u tools/bench_qrc.py 1024 >> gpurun_out/qr_ab3.log 2>&1 || exit 1
done
grep -v "n=128\|n=300" gpurun_out/qr_ab3.log
