#!/bin/bash
# Config-5 triangular solve: kernel trace + PMC passes (ordinary launches: EIGSOL_TRSV_NO_COOP=1,
# see shifted.hip).  Run from the repo root on the GPU box.
set -o pipefail
R=$(pwd); OUT=$R/gpurun_out/trsv; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export EIGSOL_TRSV_NO_COOP=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/prof_driver.py --workload config5 --steps 30 > $OUT/trace.log 2>&1 || exit 1
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_REQ_sum TCC_READ_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/pmc$i -o run -- python3 $R/tools/prof_driver.py --workload config5 --steps 30 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
cd $R
{ grep -h "sptrsv\|shift_" $OUT/trace/*kernel_stats.csv
  for d in $OUT/pmc*/; do f=$(ls $d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 tools/pmc_sum.py $f sptrsv; done; } > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
echo ok
