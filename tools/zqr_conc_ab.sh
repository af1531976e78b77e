#!/bin/bash
# A/B of the concurrent shifts (EIGSOL_ZQR_CONC / EIGSOL_QR_CONC): complex 4096^2 and 1024^2, real 4096^2
set -o pipefail
mkdir -p gpurun_out/r5
O=gpurun_out/r5/zqrconc.log
for m in 0 1 2 0 1 2; do
  EIGSOL_ZQR_CONC=$m EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qrc.py 4096 >> $O 2>&1 || exit 1
done
for m in 0 2; do
  EIGSOL_ZQR_CONC=$m timeout -k 10 120 python -u tools/bench_qrc.py 1024 >> $O 2>&1 || exit 1
done
