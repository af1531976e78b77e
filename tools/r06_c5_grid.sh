#!/bin/bash
# config 5 knob grid after the round-6 back-off / partials changes: poll mode of the role tails,
# blocks per CU per solve, head schedule, solves per launch (bench.py's config-5 leg)
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/c5_grid.log
: > $O
for rep in 1 2; do
for cfg in "" "EIGSOL_TRSV_POLL_MODE=0" "EIGSOL_TRSV_POLL_MODE=4" "EIGSOL_TRSV_POLL_MODE=6" "EIGSOL_TRSV_MULTI_HEAD=seq" "EIGSOL_TRSV_MULTI=3" "EIGSOL_TRSV_POLL_FAST=1"; do
  echo "cfg: $cfg" >> $O
  env $cfg timeout -k 10 200 python -u tools/extras_probe.py config5 2>&1 | grep -o '"ms_per_iteration": 0.[2-9][0-9]*' | head -1 >> $O || exit 1
done
done
