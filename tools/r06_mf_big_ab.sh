#!/bin/bash
# Which fronts take the row-block solve (EIGSOL_MF_BIG_NS pivots / EIGSOL_MF_BIG_D rows; shipped
# 96 / 256), after the premultiplied blocks, 1M convection-diffusion (tools/mf_probe.py), two rounds
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/mf_big_ab.log
: > $O
for r in 1 2; do
  for cfg in 96:256 64:256 128:256 192:256 96:192 96:384; do
    ns=${cfg%:*}; d=${cfg#*:}
    echo "EIGSOL_MF_BIG_NS=$ns EIGSOL_MF_BIG_D=$d" >> $O
    EIGSOL_MF_BIG_NS=$ns EIGSOL_MF_BIG_D=$d timeout -k 10 200 python -u tools/mf_probe.py 1000 >> $O 2>&1 || exit 1
  done
done
cat $O
