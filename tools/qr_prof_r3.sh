# QR kernel splits (kernel trace + stats): real 4096^2, complex 1024^2 and 4096^2.  The cooperative
# Hessenberg panel is issued by an ordinary launch (rocprofv3 crashes at exit after cooperative launches).
set -o pipefail
R=$(pwd)
mkdir -p $R/gpurun_out/qrprof
cd /tmp && export TMPDIR=/tmp
export EIGSOL_HESS_COOP_PLAIN=1
for wl in qr4096 qrc1024 qrc4096; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/qrprof/$wl -o run -- python3 $R/tools/prof_driver.py --workload $wl > $R/gpurun_out/qrprof/$wl.log 2>&1 || { echo "$wl failed"; tail -5 $R/gpurun_out/qrprof/$wl.log; exit 1; }
  echo "== $wl"; head -12 $R/gpurun_out/qrprof/$wl/run_kernel_stats.csv | cut -c1-200
done
