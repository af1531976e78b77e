#!/bin/bash
# Multifrontal solve as a replayed hipGraph vs direct launches (EIGSOL_MF_GRAPH), 1M convection-diffusion,
# alternating A/B runs in separate processes; then the multifrontal tests with the graph on.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r06_mfgraph
mkdir -p $OUT
for rep in 1 2; do
  for g in 0 1; do
    EIGSOL_MF_GRAPH=$g timeout -k 10 240 python3 -u tools/mf_probe.py 1000 > $OUT/g${g}_r${rep}.log 2>&1 || { echo "probe g=$g failed"; exit 1; }
    echo "graph=$g rep=$rep: $(tail -1 $OUT/g${g}_r${rep}.log)"
  done
done
