#!/bin/bash
# Hessenberg panel grid barrier: two-level (EIGSOL_HESS_BAR=1, default) against one counter (0),
# to_hessenberg host in/out (tools/hess_probe.py) at 1024 / 4096 / 8192, then QR 4096^2 real and complex
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/hess_bar_ab.log
: > $O
for n in 1024 4096 8192; do
  for b in 1 0 1 0; do
    echo "n $n BAR $b" >> $O
    EIGSOL_HESS_BAR=$b timeout -k 10 120 python3 tools/hess_probe.py $n >> $O 2>&1 || exit 1
  done
done
for b in 1 0; do
  echo "QR BAR $b" >> $O
  EIGSOL_HESS_BAR=$b timeout -k 10 120 python3 -u tools/bench_qr.py 4096 >> $O 2>&1 || exit 1
  EIGSOL_HESS_BAR=$b timeout -k 10 120 python3 -u tools/bench_qrc.py 4096 >> $O 2>&1 || exit 1
done
