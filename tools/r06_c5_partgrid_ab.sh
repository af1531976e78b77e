#!/bin/bash
# config 5: the partials / move-out kernel's grid (EIGSOL_TRSV_PART_GRID), bench.py's own config-5 leg
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/c5_partgrid_ab2.log
: > $O
for g in 256 128 64 192 256 128 64 192; do
  echo "EIGSOL_TRSV_PART_GRID=$g" >> $O
  EIGSOL_TRSV_PART_GRID=$g timeout -k 10 200 python -u tools/extras_probe.py config5 2>&1 | grep -o '"ms_per_iteration": 0.[2-9][0-9]*' >> $O || exit 1
done
