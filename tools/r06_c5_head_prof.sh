#!/bin/bash
# config 5 head / tail / partials split per K (kernel trace; ordinary launches, EIGSOL_TRSV_NO_COOP=1,
# as tools/trsv_prof.sh: the profiler and cooperative launches do not mix), and the L2 hit rate
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/r6/c5prof; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export EIGSOL_TRSV_NO_COOP=1
for K in 4 1 2; do
  EIGSOL_TRSV_MULTI=$K timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/k$K -o run -- python3 $R/tools/prof_driver.py --workload config5 --steps 20 > $OUT/k$K.log 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --output-format csv -d $OUT/pmc -o run -- python3 $R/tools/prof_driver.py --workload config5 --steps 20 > $OUT/pmc.log 2>&1
