#!/bin/bash
# Config-5 shifted inverse iteration: kernel traces with one and with K = 4 reference iterations
# per launch (ordinary launches, EIGSOL_TRSV_NO_COOP=1).  Run from the repo root on the GPU box.
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/multi; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export EIGSOL_TRSV_NO_COOP=1
for k in ${TRSV_KS:-1 4}; do
  EIGSOL_TRSV_MULTI=$k timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace$k -o run -- python3 $R/tools/prof_driver.py --workload config5 --steps 30 > $OUT/trace$k.log 2>&1 || exit 1
  python3 $R/tools/prof_stats.py $OUT/trace$k > $OUT/stats$k.txt
done
echo ok
