#!/bin/bash
# Hessenberg panel with value flags (hess_panel_coop3, EIGSOL_HESS_VAL=1, default) against two grid barriers per
# (the value-flag panel, EIGSOL_HESS_VAL, was measured slower and removed; the script documents profiles/r06_hess_val_ab.log)
# column (hess_panel_coop2, EIGSOL_HESS_VAL=0): to_hessenberg host in/out at 1024 / 4096 / 8192, QR 4096^2 real / complex
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/hess_val_ab.log
: > $O
for n in 1024 4096 8192; do
  for v in 1 0 1 0; do
    echo "n $n VAL $v" >> $O
    EIGSOL_HESS_VAL=$v timeout -k 10 120 python3 tools/hess_probe.py $n >> $O 2>&1 || exit 1
  done
done
for v in 1 0; do
  echo "QR VAL $v" >> $O
  EIGSOL_HESS_VAL=$v timeout -k 10 120 python3 -u tools/bench_qr.py 4096 >> $O 2>&1 || exit 1
  EIGSOL_HESS_VAL=$v timeout -k 10 120 python3 -u tools/bench_qrc.py 4096 >> $O 2>&1 || exit 1
done
