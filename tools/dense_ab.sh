#!/bin/bash
# Dense GEMV: split-row 8-byte loads x blocks per CU target (tools/dense_ab.py, one process each).
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/dense_ab.log
for split in 0 1; do
  for tgt in 2048 1024 512; do
    EIGSOL_DENSE_SPLIT=$split EIGSOL_DENSE_TARGET=$tgt timeout -k 10 150 python -u tools/dense_ab.py >> gpurun_out/dense_ab.log 2>&1 || exit 1
  done
done
