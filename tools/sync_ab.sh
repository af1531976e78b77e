#!/bin/bash
# A/B of the host wait in host-driven loops (EIGSOL_SYNC_SPIN=0: hipStreamSynchronize; 1: spin on
# hipStreamQuery): real / complex QR 4096^2 and the GMRES shifted iteration; then a kernel trace of
# the real QR with its idle-gap analysis.  Run on the GPU box from the repo root.
set -e
mkdir -p gpurun_out/sync_ab
for v in 0 1; do
  EIGSOL_SYNC_SPIN=$v timeout -k 10 120 python -u tools/bench_qr.py 4096 > gpurun_out/sync_ab/qr_$v.log 2>&1
  EIGSOL_SYNC_SPIN=$v timeout -k 10 120 python -u tools/bench_qrc.py 4096 > gpurun_out/sync_ab/qrc_$v.log 2>&1
  EIGSOL_SYNC_SPIN=$v timeout -k 10 200 python -u tools/gmres_warm_ab.py > gpurun_out/sync_ab/gmres_$v.log 2>&1
  EIGSOL_GMRES_WARM=0 EIGSOL_SYNC_SPIN=$v timeout -k 10 200 python -u tools/gmres_warm_ab.py > gpurun_out/sync_ab/gmres_cold_$v.log 2>&1
done
ROOTD=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd $ROOTD
EIGSOL_HESS_COOP_PLAIN=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sync_ab/qr_trace -o run -- python3 tools/bench_qr.py 4096 > gpurun_out/sync_ab/qr_trace.log 2>&1
python3 tools/gap_analysis.py gpurun_out/sync_ab/qr_trace/run_kernel_trace.csv > gpurun_out/sync_ab/qr_gaps.txt 2>&1
EIGSOL_HESS_COOP_PLAIN=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sync_ab/qrc_trace -o run -- python3 tools/bench_qrc.py 4096 > gpurun_out/sync_ab/qrc_trace.log 2>&1
python3 tools/gap_analysis.py gpurun_out/sync_ab/qrc_trace/run_kernel_trace.csv > gpurun_out/sync_ab/qrc_gaps.txt 2>&1
rm -rf gpurun_out/sync_ab/qr_trace gpurun_out/sync_ab/qrc_trace
