#!/bin/bash
# A/B of library variants on the headline workload: tools/ab_bench.sh lib1.so lib2.so ...
set -o pipefail
for lib in "$@"; do
  echo "== $lib"
  EIGSOL_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --steps 200 --warmup 20 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['event_ms_per_launch'], d['roofline']['frac'])" || exit 1
done
