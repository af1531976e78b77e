#!/bin/bash
# f64 MFMA GEMM K-step (EIGSOL_GEMM_KT 16 / 32 / 64): kernel trace of to_hessenberg 4096^2 (tools/hess_prof.sh),
# (the EIGSOL_GEMM_KT switch was measured flat and removed; the script documents profiles/r06_gemm_kt_ab.log)
# summed GEMM kernel time of the last reduction, then QR 4096^2 (tools/bench_qr.py)
set -o pipefail
mkdir -p gpurun_out/r6
O=gpurun_out/r6/gemm_kt_ab.log
: > $O
for kt in ${KTS:-16 32 64}; do
  echo "== KT $kt" >> $O
  EIGSOL_GEMM_KT=$kt tools/hess_prof.sh pcsc_eigenvalue_solver_project_amd/libeigsol_hip.so >> $O 2>&1 || exit 1
  python3 - gpurun_out/hessprof1/run_kernel_trace.csv >> $O <<'PY'
import csv, sys, collections
t = [r for r in csv.DictReader(open(sys.argv[1]))]
half = len(t) // 2     # the second of the probe's timed reductions
agg = collections.defaultdict(lambda: [0, 0.0])
for r in t[half:]:
    k = r['Kernel_Name'].split('(')[0][:70]
    agg[k][0] += 1
    agg[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:8]:
    print(f"  {v[1]:8.2f} ms {v[0]:5d}  {k}")
PY
  EIGSOL_GEMM_KT=$kt timeout -k 10 120 python3 -u tools/bench_qr.py 4096 >> $O 2>&1 || exit 1
done
