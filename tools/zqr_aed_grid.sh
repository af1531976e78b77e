#!/bin/bash
# Complex QR: AED window x nibble grid at 1024^2 and 4096^2 (one process per point: the knobs are read once)
set -o pipefail
for n in 1024 4096; do
  for w in 48 56 64; do
    for nib in 14 25; do
      EIGSOL_ZQR_AED=$w EIGSOL_ZQR_NIBBLE=$nib timeout -k 10 100 python3 tools/bench_qrc.py $n || exit 1
    done
  done
done
