#!/bin/bash
# Round-6 headline evidence (on the GPU box, from the repo root): the bench line (with the 12:1
# read/write probe), the kernel-trace summary of the same command, and the FETCH_SIZE / WRITE_SIZE
# passes of the shipped instantiation (each pass its own run, never combined with trace domains).
set -o pipefail
R=$(pwd)
OUT=$R/gpurun_out/r06_headline
mkdir -p $OUT
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-extras --steps 200 --warmup 20 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-extras --no-cpu-baseline --steps 200 --warmup 20 > $OUT/trace.log 2>&1 || { echo "trace failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc1 -o run -- python3 $R/tools/prof_driver.py --workload band10m --steps 20 > $OUT/pmc1.log 2>&1 || { echo "pmc1 failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc2 -o run -- python3 $R/tools/prof_driver.py --workload band10m --steps 20 > $OUT/pmc2.log 2>&1 || { echo "pmc2 failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $OUT/pmc3 -o run -- python3 $R/tools/prof_driver.py --workload band10m --steps 20 > $OUT/pmc3.log 2>&1 || { echo "pmc3 failed"; exit 1; }
echo "headline profile ok"
