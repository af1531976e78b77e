#!/bin/bash
# Config-5 pair launches: timing variants, then kernel traces of one solve per launch vs pair
# launches (ordinary launches, EIGSOL_TRSV_NO_COOP=1).  Run from the repo root on the GPU box.
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/pair; mkdir -p $OUT
timeout -k 10 300 python3 -u $R/tools/trsv_variants.py "EIGSOL_TRSV_PAIR=0" "EIGSOL_TRSV_PAIR=2" \
  "EIGSOL_TRSV_PAIR=2 EIGSOL_TRSV_POLL_FAST=64" "EIGSOL_TRSV_PAIR=1 EIGSOL_TRSV_POLL_FAST=64" \
  "EIGSOL_TRSV_PAIR=0 EIGSOL_TRSV_POLL_FAST=64" "EIGSOL_TRSV_PAIR=2 EIGSOL_TRSV_BLOCKS_PER_CU=1" \
  "EIGSOL_TRSV_PAIR=1 EIGSOL_TRSV_BLOCKS_PER_CU=3" > $OUT/variants.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
export EIGSOL_TRSV_NO_COOP=1
for p in 0 2; do
  EIGSOL_TRSV_PAIR=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace$p -o run -- python3 $R/tools/prof_driver.py --workload config5 --steps 30 > $OUT/trace$p.log 2>&1 || exit 1
  python3 $R/tools/prof_stats.py $OUT/trace$p > $OUT/stats$p.txt
done
echo ok
