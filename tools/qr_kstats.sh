#!/bin/bash
# per-kernel stats of the 4096^2 QR for each library given: tools/qr_kstats.sh lib1.so lib2.so ...
# (EIGSOL_HESS_NO_COOP: rocprofv3 crashes at exit after a cooperative launch on this image)
set -o pipefail
R=$(pwd)
i=0
for lib in "$@"; do
  i=$((i + 1))
  OUT=$R/gpurun_out/qrk$i
  mkdir -p $OUT
  (cd /tmp && export TMPDIR=/tmp && EIGSOL_LIB_PATH=$R/$lib EIGSOL_HESS_NO_COOP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/tools/prof_driver.py --workload qr4096 > $OUT.log 2>&1) || exit 1
  echo "== $lib"
  python3 - $OUT/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(f"{r['Name'][:50]:50s} {int(r['Calls']):7d} {float(r['TotalDurationNs'])/1e6:9.1f} ms {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
