#!/bin/bash
# config 5 tail back-off A/B (EIGSOL_TRSV_POLL_SLOW: the re-poll sleep schedule, shifted.hip
# poll_backoff; EIGSOL_TRSV_POLL_FAST: re-polls without a sleep first), bench.py's own config-5 leg
# (tools/extras_probe.py config5)
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/trsv_backoff_ab3.log
: > $O
for cfg in "0 0" "1 0" "2 0" "4 0" "4 1" "4 2" "6 0" "0 0" "1 0" "2 0" "4 0" "4 1" "4 2" "6 0"; do
  set -- $cfg
  echo "EIGSOL_TRSV_POLL_SLOW=$1 EIGSOL_TRSV_POLL_FAST=$2" >> $O
  EIGSOL_TRSV_POLL_SLOW=$1 EIGSOL_TRSV_POLL_FAST=$2 timeout -k 10 200 python -u tools/extras_probe.py config5 2>&1 | grep -o '"ms_per_iteration": 0.[2-9][0-9]*' >> $O || exit 1
done
