#!/bin/bash
# General-sparse shifted inverse (ILU(0) + GMRES, 1M): kernel trace with ordinary launches.
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/gmres; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export EIGSOL_TRSV_NO_COOP=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/prof_driver.py --workload gmres1m --steps 4 > $OUT/trace.log 2>&1 || exit 1
python3 $R/tools/prof_stats.py $OUT/trace > $OUT/stats.txt
echo ok
