#!/bin/bash
# Round GPU pass (from the repo root on the GPU box): every GPU test, the default bench line, and
# the kernel-trace summary of the headline bench command.  Each step has its own time limit; the
# script stops at the first failure.
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/round
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/gputest.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/headline -o run -- python3 $R/bench.py --no-extras --no-cpu-baseline > $OUT/headline.log 2>&1 || { echo "headline profile failed"; exit 1; }
echo "round pass ok"
