#!/bin/bash
# complex QR: in-tree build against candidate builds tools/ab/libeigsol_z*.so (bitwise + time)
set -o pipefail
OUT=gpurun_out/zab; mkdir -p $OUT
export QR_AB_SIZES=-64,-200,-1024
timeout -k 10 120 python -u tools/qr_ab.py $OUT/tree.npz || exit 1
for v in zA zB; do
  EIGSOL_LIB_PATH=$PWD/tools/ab/libeigsol_$v.so timeout -k 10 120 python -u tools/qr_ab.py $OUT/$v.npz || exit 1
done
timeout -k 10 120 python -u tools/qr_ab.py $OUT/tree2.npz || exit 1
python - <<'PY'
import numpy as np
t = np.load("gpurun_out/zab/tree.npz")
for v in ("zA", "zB", "tree2"):
    a = np.load(f"gpurun_out/zab/{v}.npz")
    print(v, {k: (a[k].tobytes() == t[k].tobytes()) if k.startswith("ev") else round(float(a[k]), 4) for k in a.files}, flush=True)
print("tree", {k: round(float(t[k]), 4) for k in t.files if k.startswith("t")})
PY
