#!/bin/bash
# Real 4096^2 QR at nibble 15: bulges x AED window, two seeds.  Output: gpurun_out/qr_grid_r5b.log
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/qr_grid_r5b.log
: > $OUT
for seed in 42 7; do
  for nb in 28 32 36; do
    for aed in 56 64 72; do
      echo "== seed $seed nb $nb aed $aed" >> $OUT
      QR_SEED=$seed EIGSOL_QR_NB=$nb EIGSOL_QR_AED=$aed timeout -k 10 120 python -u tools/bench_qr.py 4096 2>/dev/null | grep seconds >> $OUT || exit 1
    done
  done
done
cat $OUT
