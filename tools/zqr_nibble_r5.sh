#!/bin/bash
# Complex 4096^2 / 1024^2 QR: AED nibble.  Output: gpurun_out/zqr_nibble_r5.log
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/zqr_nibble_r5.log
: > $OUT
for n in 4096 1024; do
  for nib in 14 10 20 7; do
    echo "== n $n nibble $nib" >> $OUT
    EIGSOL_ZQR_NIBBLE=$nib timeout -k 10 120 python -u tools/bench_qrc.py $n 2>/dev/null | grep "eigvals/s" >> $OUT || exit 1
  done
done
cat $OUT
