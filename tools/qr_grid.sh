#!/bin/bash
# QR 4096 wall time over the Francis tuning knobs: tools/qr_grid.sh "AED NB GROUPS NIBBLE" ...
for cfg in "$@"; do
  set -- $cfg
  r=$(EIGSOL_QR_AED=$1 EIGSOL_QR_NB=$2 EIGSOL_QR_GROUPS=$3 EIGSOL_QR_NIBBLE=$4 EIGSOL_QR_STATS=1 timeout -k 10 60 python tools/bench_qr.py 2>&1) || { echo "$cfg FAILED"; echo "$r" | tail -3; exit 1; }
  echo "aed=$1 nb=$2 groups=$3 nibble=$4 :: $(echo "$r" | grep 'n=4096' | sed 's/.*sweeps=\([0-9]*\) windows=\([0-9]*\) steps=\([0-9]*\).*aed=\([0-9]*\) aed_deflated.*/sweeps=\1 windows=\2 steps=\3 aed=\4/') :: $(echo "$r" | tail -1 | python3 -c 'import json,sys; d=json.load(sys.stdin); print(round(d["seconds"],3), d["converged"], d["max_match_dist"])')"
done
