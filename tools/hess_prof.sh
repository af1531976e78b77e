#!/bin/bash
# Kernel-trace the blocked Hessenberg (4096^2, the panel through an ordinary launch) for each library
# and print the summed panel time of the last reduction:  tools/hess_prof.sh lib1.so lib2.so ...
set -o pipefail
R=$(pwd)
i=0
for lib in "$@"; do
  i=$((i + 1))
  OUT=$R/gpurun_out/hessprof$i
  mkdir -p $OUT
  (cd /tmp && export TMPDIR=/tmp && EIGSOL_LIB_PATH=$R/$lib EIGSOL_HESS_COOP_PLAIN=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 $R/tools/hess_probe.py 4096 > $OUT.log 2>&1) || exit 1
  python3 - $OUT/run_kernel_trace.csv $lib <<'PY'
import csv, sys
t = [r for r in csv.DictReader(open(sys.argv[1]))]
p = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in t if 'hess_panel_coop' in r['Kernel_Name']]
allk = sum((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in t)
print(f"{sys.argv[2]}: panels (last 128) {sum(p[-128:]):.2f} ms, previous 128 {sum(p[-256:-128]):.2f} ms")
PY
done
