#!/bin/bash
# per-workload A/B: tools/ab_workloads.sh "band1m uniform1m" lib1.so lib2.so ...
set -o pipefail
wls=$1; shift
for wl in $wls; do
  for lib in "$@"; do
    printf "%-10s %-50s " $wl $lib
    EIGSOL_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --workload $wl --steps 400 --warmup 20 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['roofline']['event_ms_per_launch'], d['roofline']['frac'])" || exit 1
  done
done
