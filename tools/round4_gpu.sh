#!/bin/bash
# Round-4 GPU pass (repo root on the GPU box). Part "a": every GPU test, the default bench line,
# the headline kernel trace; part "b": QR kernel splits (4096^2 real with the cooperative panel
# issued as an ordinary launch, rocprofv3 crashes after cooperative launches; 4096^2 complex) and
# the uniform10m binned-kernel trace + FETCH/WRITE PMC passes.  Stops at the first failure.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r4
mkdir -p $OUT
part=${1:-a}
if [ "$part" = a ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || { echo "gpu tests failed"; exit 1; }
  timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; exit 1; }
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/headline -o run -- python3 $R/bench.py --no-extras --no-cpu-baseline > $OUT/headline.log 2>&1 || { echo "headline profile failed"; exit 1; }
  echo "part a ok"
elif [ "$part" = q ]; then
  cd /tmp && export TMPDIR=/tmp
  EIGSOL_HESS_COOP_PLAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/qr4096 -o run -- python3 $R/tools/prof_driver.py --workload qr4096 > $OUT/qr4096.log 2>&1 || { echo "qr4096 profile failed"; exit 1; }
  EIGSOL_HESS_COOP_PLAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/qrc4096 -o run -- python3 $R/tools/prof_driver.py --workload qrc4096 > $OUT/qrc4096.log 2>&1 || { echo "qrc4096 profile failed"; exit 1; }
  echo "part q ok"
else
  cd /tmp && export TMPDIR=/tmp
  EIGSOL_HESS_COOP_PLAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/qr4096 -o run -- python3 $R/tools/prof_driver.py --workload qr4096 > $OUT/qr4096.log 2>&1 || { echo "qr4096 profile failed"; exit 1; }
  EIGSOL_HESS_COOP_PLAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/qrc4096 -o run -- python3 $R/tools/prof_driver.py --workload qrc4096 > $OUT/qrc4096.log 2>&1 || { echo "qrc4096 profile failed"; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/uni -o run -- python3 $R/tools/prof_driver.py --workload uniform10m --steps 20 > $OUT/uni.log 2>&1 || { echo "uniform trace failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/uni_fetch -o run -- python3 $R/tools/prof_driver.py --workload uniform10m --steps 20 > $OUT/uni_fetch.log 2>&1 || { echo "uniform fetch failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/uni_write -o run -- python3 $R/tools/prof_driver.py --workload uniform10m --steps 20 > $OUT/uni_write.log 2>&1 || { echo "uniform write failed"; exit 1; }
  cd $R
  EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qr.py 4096 > $OUT/qr_time.log 2>&1 || { echo "qr timing failed"; exit 1; }
  EIGSOL_QR_STATS=1 timeout -k 10 120 python -u tools/bench_qrc.py 4096 > $OUT/qrc_time.log 2>&1 || { echo "qrc timing failed"; exit 1; }
  echo "part b ok"
fi
