#!/bin/bash
# Hessenberg panel grid (EIGSOL_HESS_G blocks, one 1024-thread block per CU): to_hessenberg 4096^2 host in/out
# (tools/hess_probe.py) and QR 4096^2 real / complex (tools/bench_qr.py, tools/bench_qrc.py) per grid size
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/hess_grid_ab.log
: > $O
for g in ${GRIDS:-64 128 256 128 64 256}; do
  echo "== G $g" >> $O
  EIGSOL_HESS_G=$g timeout -k 10 120 python3 tools/hess_probe.py 4096 >> $O 2>&1 || exit 1
done
for g in ${QRGRIDS:-64 128 256}; do
  echo "== QR G $g" >> $O
  EIGSOL_HESS_G=$g timeout -k 10 120 python3 -u tools/bench_qr.py 4096 >> $O 2>&1 || exit 1
  EIGSOL_HESS_G=$g timeout -k 10 120 python3 -u tools/bench_qrc.py 4096 >> $O 2>&1 || exit 1
done
