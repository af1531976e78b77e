#!/bin/bash
# Real 4096^2 QR after the round-5 concurrent shifts (EIGSOL_QR_CONC=2): bulges x AED window x nibble,
# two seeds.  Run from the repo root on the GPU box.  Output: gpurun_out/qr_grid_r5.log
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/qr_grid_r5.log
: > $OUT
for seed in 42 7; do
  for cfg in ${QR_GRID_CFGS:-"EIGSOL_QR_NB=32 EIGSOL_QR_AED=64" "EIGSOL_QR_NB=28 EIGSOL_QR_AED=64" "EIGSOL_QR_NB=40 EIGSOL_QR_AED=64"} \
             "EIGSOL_QR_NB=32 EIGSOL_QR_AED=80" "EIGSOL_QR_NB=40 EIGSOL_QR_AED=80" "EIGSOL_QR_NB=32 EIGSOL_QR_AED=64 EIGSOL_QR_NIBBLE=20" \
             "EIGSOL_QR_NB=32 EIGSOL_QR_AED=64 EIGSOL_QR_NIBBLE=40"; do
    echo "== seed $seed $cfg" >> $OUT
    env QR_SEED=$seed $cfg timeout -k 10 120 python -u tools/bench_qr.py 4096 2>/dev/null | grep seconds >> $OUT || exit 1
  done
done
cat $OUT
