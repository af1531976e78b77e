#!/bin/bash
# Real 4096^2 QR: AED nibble (skip the sweep when the AED deflated more than this % of its window), two
# seeds, after the round-5 concurrent shifts.  Output: gpurun_out/qr_nibble_r5.log
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/qr_nibble_r5.log
: > $OUT
for seed in 42 7 20251226; do
  for nib in 30 25 20 15 10; do
    echo "== seed $seed nibble $nib" >> $OUT
    QR_SEED=$seed EIGSOL_QR_NIBBLE=$nib timeout -k 10 120 python -u tools/bench_qr.py 4096 2>/dev/null | grep seconds >> $OUT || exit 1
  done
done
cat $OUT
