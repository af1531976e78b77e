#!/bin/bash
# kernel stats of the 4096^2 QR at several bulge-group counts
set -o pipefail
ROOTD=$(pwd)
OUT=$ROOTD/gpurun_out/qrg
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for g in ${GROUPS_LIST:-1 4}; do
  EIGSOL_QR_GROUPS=$g EIGSOL_HESS_NO_COOP=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/g$g -o run -- python3 $ROOTD/tools/prof_driver.py --workload qr4096 > $OUT/g$g.log 2>&1 || exit 1
  python3 - $OUT/g$g/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:50]:50s} {int(r['Calls']):7d} {float(r['TotalDurationNs'])/1e6:9.1f} ms {float(r['AverageNs'])/1e3:9.1f} us")
PY
done
