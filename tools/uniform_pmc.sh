#!/bin/bash
# Config 3 (uniform1m) line-traffic evidence: kernel trace, then one rocprofv3 --pmc pass per counter
# group (never combined with trace domains).  Output: gpurun_out/upmc/*, summary gpurun_out/upmc/summary.txt
set -o pipefail
ROOTD=$(pwd)
OUT=$ROOTD/gpurun_out/upmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $ROOTD/tools/prof_driver.py --workload uniform1m --steps 20 > $OUT/trace.log 2>&1 || exit 1
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TA_BUSY_avr TA_TA_BUSY_sum" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/pmc$i -o run -- python3 $ROOTD/tools/prof_driver.py --workload uniform1m --steps 20 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($ctrs) failed" >> $OUT/errors.log; exit 1; }
done
cd $ROOTD
{ grep -h "csr_" $OUT/trace/*kernel_stats.csv | head -5
  for d in $OUT/pmc*/; do f=$(ls $d/*counter_collection.csv 2>/dev/null | head -1); [ -n "$f" ] && python3 tools/pmc_sum.py $f csr_; done; } > $OUT/summary.txt 2>&1
cat $OUT/summary.txt
