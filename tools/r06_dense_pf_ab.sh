#!/bin/bash
# Dense shifted inverse: dense_trsv2_kernel with the tile loads one block ahead (1) and the premultiplied next-to-diagonal block (2, default) against the
# unpipelined loop (EIGSOL_DENSE_PF=0), two rounds.  Output: gpurun_out/r6/dense_pf_ab.log
set -o pipefail
mkdir -p gpurun_out/r6
OUT=gpurun_out/r6/dense_pf_ab.log
: > $OUT
for r in 1 2; do
  for pf in 2 1 0; do
    echo "== EIGSOL_DENSE_PF=$pf" >> $OUT
    EIGSOL_DENSE_PF=$pf timeout -k 10 240 python -u tools/bench_dense_shifted.py 8192:f64 16384:f64 8192:c128 16384:c128 32768:f64 2>/dev/null >> $OUT || exit 1
  done
done
cat $OUT
