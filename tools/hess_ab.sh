#!/bin/bash
# A/B of the blocked Hessenberg reduction (host in/out) over variant libraries:
#   tools/hess_ab.sh build/var/lib_a.so build/var/lib_b.so ...   (n = 4096; EIGSOL_HESS_N overrides)
set -o pipefail
n=${EIGSOL_HESS_N:-4096}
for lib in "$@"; do
  echo "== $lib"
  EIGSOL_LIB_PATH=$lib timeout -k 10 120 python3 tools/hess_probe.py $n || exit 1
done
