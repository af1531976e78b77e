#!/bin/bash
# QR kernel splits as shipped (on the GPU box, from the repo root): config 2 (4096^2 real) with the
# cooperative Hessenberg panel issued through an ordinary launch (EIGSOL_HESS_COOP_PLAIN=1: the same
# kernel; rocprofv3 crashes after cooperative launches), and the complex 1024^2 QR.
set -o pipefail
R=$(pwd)
OUT=$R/${1:-gpurun_out/qrprof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
EIGSOL_HESS_COOP_PLAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/qr4096 -o run -- python3 $R/tools/prof_driver.py --workload qr4096 > $OUT/qr4096.log 2>&1 || { echo "qr4096 profile failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/qrc1024 -o run -- python3 $R/tools/prof_driver.py --workload qrc1024 > $OUT/qrc1024.log 2>&1 || { echo "qrc1024 profile failed"; exit 1; }
echo "qr profiles ok"
