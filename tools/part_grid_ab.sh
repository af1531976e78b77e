#!/bin/bash
# Config 5 multi-solve: the partials kernel's grid (EIGSOL_TRSV_PART_GRID) -> ms per iteration.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/part_grid.log
for g in 1024 2048 512 1024; do
  EIGSOL_TRSV_PART_GRID=$g timeout -k 10 200 python -u tools/bench_shifted.py >> gpurun_out/part_grid.log 2>&1 || exit 1
done
