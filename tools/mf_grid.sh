#!/bin/bash
# Multifrontal solve knobs on the 1M convection-diffusion matrix (tools/mf_probe.py): leaf size,
# large-front thresholds, flag back-off.  Output: gpurun_out/mf_grid.log
cd "$(dirname "$0")/.." || exit 1
OUT=gpurun_out/mf_grid.log
: > $OUT
run() { echo "== $*" >> $OUT; env "$@" timeout -k 10 120 python -u tools/mf_probe.py 1000 >> $OUT 2>&1 || exit 1; }
run EIGSOL_MF_BACKOFF=1
run EIGSOL_MF_BACKOFF=0
run EIGSOL_MF_LEAF=32
run EIGSOL_MF_LEAF=128
run EIGSOL_MF_BIG_NS=96 EIGSOL_MF_BIG_D=384
run EIGSOL_MF_BIG_NS=192 EIGSOL_MF_BIG_D=768
