#!/bin/bash
# Usage (on the GPU box, from the repo root): tools/profile.sh <outdir> [workload] [steps]
# 1) kernel trace + stats; 2) separate PMC passes (never combined with trace domains).
set -o pipefail
OUT=${1:-gpurun_out/prof}; WL=${2:-band10m}; ST=${3:-20}
ROOTD=$(pwd)
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOTD/$OUT/trace -o run -- python3 $ROOTD/tools/prof_driver.py --workload $WL --steps $ST > $ROOTD/$OUT/trace.log 2>&1 || exit 1
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr TA_TA_BUSY_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d $ROOTD/$OUT/pmc$i -o run -- python3 $ROOTD/tools/prof_driver.py --workload $WL --steps $ST > $ROOTD/$OUT/pmc$i.log 2>&1 || echo "pmc pass $i ($ctrs) failed" >> $ROOTD/$OUT/errors.log
done
exit 0
