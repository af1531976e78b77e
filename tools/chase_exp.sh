#!/bin/bash
# QR chase experiment: per-step chase time at several bulge counts (rocprofv3 kernel stats + EIGSOL_QR_STATS)
set -o pipefail
ROOTD=$(pwd)
OUT=$ROOTD/gpurun_out/chase
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for nb in ${NBS:-16 8 4}; do
  EIGSOL_QR_STATS=1 EIGSOL_QR_NB=$nb EIGSOL_HESS_NO_COOP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/nb$nb -o run -- python3 $ROOTD/tools/prof_driver.py --workload qr4096 > $OUT/nb$nb.log 2>&1 || exit 1
  grep "francis:" $OUT/nb$nb.log
  grep -h "chase\|aed_kernel\|win_gemm" $OUT/nb$nb/run_kernel_stats.csv | cut -d, -f1-4
done
