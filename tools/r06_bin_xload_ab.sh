#!/bin/bash
# uniform-column SpMV (csr_bin_kernel): the x gathers' load flavour, A/B builds in ab/ (EIGSOL_LIB_PATH):
# plain (the shipped library), non-temporal, agent-scope; bench.py --workload uniform1m / uniform10m
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/bin_xload_ab.log
: > $O
for rep in 1 2; do
for lib in "" "$PWD/ab/lib_x1.so" "$PWD/ab/lib_x2.so"; do
  for w in uniform1m uniform10m; do
    echo "lib=${lib:-shipped} workload=$w" >> $O
    EIGSOL_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --workload $w --no-extras --no-cpu-baseline --steps 100 --warmup 10 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> $O || exit 1
  done
done
done
