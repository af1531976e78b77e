#!/bin/bash
# Round-6 QR kernel splits of the shipped path (on the GPU box, from the repo root): config 2
# (4096^2 real, cooperative Hessenberg panel issued through an ordinary launch of the same kernel,
# EIGSOL_HESS_COOP_PLAIN=1: rocprofv3 crashes after cooperative launches) and the complex 4096^2 QR.
set -o pipefail
R=$(pwd)
OUT=$R/${1:-gpurun_out/r06qr}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
EIGSOL_HESS_COOP_PLAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/qr4096 -o run -- python3 $R/tools/prof_driver.py --workload qr4096 > $OUT/qr4096.log 2>&1 || { echo "qr4096 profile failed"; exit 1; }
EIGSOL_HESS_COOP_PLAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/qrc4096 -o run -- python3 $R/tools/prof_driver.py --workload qrc4096 > $OUT/qrc4096.log 2>&1 || { echo "qrc4096 profile failed"; exit 1; }
echo "qr profiles ok"
