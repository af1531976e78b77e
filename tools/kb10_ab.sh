#!/bin/bash
# A/B: band10m headline with KB = 10 (five value loads per lane) against KB = 12
set -o pipefail
mkdir -p gpurun_out/r5
O=gpurun_out/r5/kb10.log
for r in 1 2 3; do
  for m in 0 1; do
    EIGSOL_SLICE_KB10=$m timeout -k 10 200 python -u bench.py --no-extras --no-cpu-baseline --steps 200 > gpurun_out/r5/kb10_one.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/r5/kb10_one.log').read().strip().splitlines()[-1]); print('KB10=$m', d['roofline']['kernel'][:70], d['roofline']['event_ms_per_launch'], d['value'])" >> $O
  done
done
