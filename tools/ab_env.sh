#!/bin/bash
# A/B over env settings: tools/ab_env.sh lib.so "VAR=val ..." "VAR=val ..."
set -o pipefail
lib=$1; shift
for e in "$@"; do
  echo "== $lib $e"
  env $e EIGSOL_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --steps 200 --warmup 20 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['roofline']['event_ms_per_launch'], d['roofline']['frac'])" || exit 1
done
