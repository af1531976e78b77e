#!/bin/bash
# Dense power GEMV: columns per load batch (EIGSOL_DENSE_KU 8 shipped, variants 4 / 12 / 16) and the
# 8-byte split-row loads, 16384^2 f64 / c128, two rounds.  Output: gpurun_out/r6/dense_ku_ab.log
set -o pipefail
mkdir -p gpurun_out/r6
OUT=gpurun_out/r6/dense_ku_ab.log
: > $OUT
for r in 1 2; do
  for v in ship ku4 ku12 ku16 split; do
    echo "== $v" >> $OUT
    L=""; [ "$v" != ship ] && [ "$v" != split ] && L=build/var/lib_$v.so
    S=0; [ "$v" = split ] && S=1
    EIGSOL_LIB_PATH=$L EIGSOL_DENSE_SPLIT=$S timeout -k 10 200 python -u tools/bench_dense_power.py 16384:f64 16384:c128 2>/dev/null >> $OUT || exit 1
  done
done
cat $OUT
