#!/bin/bash
# A/B of a candidate library (tools/ab/libeigsol_qrlat.so) against the in-tree build: QR eigenvalues
# (bitwise where the change is meant to be exact) and times, the QR GPU tests on the candidate, and
# the band10m power-iteration probe (in-tree vs pre-segmentation build).
set -o pipefail
OUT=gpurun_out/qrab
mkdir -p $OUT
CAND=$PWD/tools/ab/libeigsol_qrlat.so
timeout -k 10 200 python -u tools/qr_ab.py $OUT/old.npz || exit 1
EIGSOL_LIB_PATH=$CAND timeout -k 10 200 python -u tools/qr_ab.py $OUT/new.npz || exit 1
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/qrab/new.npz"); b = np.load("gpurun_out/qrab/old.npz")
for k in a.files:
    print(k, (a[k].tobytes() == b[k].tobytes()) if k.startswith("ev") else (float(a[k]), float(b[k])), flush=True)
PY
EIGSOL_LIB_PATH=$CAND timeout -k 10 300 python -u -m pytest tests/test_gpu_qr.py tests/test_gpu_fullsize.py -k "qr or francis or hessenberg" -x -q --timeout 120 --timeout-method thread > $OUT/qrtests.log 2>&1 || { tail -30 $OUT/qrtests.log; echo "qr tests failed"; exit 1; }
tail -2 $OUT/qrtests.log
timeout -k 10 120 python -u tools/ab_probe.py || exit 1
EIGSOL_LIB_PATH=$PWD/tools/ab/libeigsol_preseg.so timeout -k 10 120 python -u tools/ab_probe.py || exit 1
timeout -k 10 120 python -u tools/ab_probe.py || exit 1
echo "qrlat pass ok"
