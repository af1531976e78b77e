#!/bin/bash
# Multifrontal solve knobs on the 1M convection-diffusion matrix (tools/mf_probe.py): leaf size,
# large-front thresholds, flag back-off / acquire mode.  Output: gpurun_out/mf_grid.log
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/mf_grid.log
: > $OUT
run() { echo "== $*" >> $OUT; env "$@" timeout -k 10 120 python -u tools/mf_probe.py 1000 >> $OUT 2>&1 || exit 1; }
if [ $# -gt 0 ]; then for cfg in "$@"; do run $cfg; done; exit 0; fi
run EIGSOL_MF_BACKOFF=0
run EIGSOL_MF_BACKOFF=2
run EIGSOL_MF_BACKOFF=2 EIGSOL_MF_BIG_NS=64 EIGSOL_MF_BIG_D=256
run EIGSOL_MF_BACKOFF=2 EIGSOL_MF_BIG_NS=48 EIGSOL_MF_BIG_D=192
