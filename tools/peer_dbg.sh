#!/bin/bash
# single-precision peer debugging + column-block default check
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/peer_single_debug.py > gpurun_out/peer_dbg.log 2>&1; rc=$?
cat gpurun_out/peer_dbg.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -m pytest tests/test_gpu_power.py -k column_blocked -q --timeout 120 --timeout-method thread > gpurun_out/cblk_tests2.log 2>&1 && tail -2 gpurun_out/cblk_tests2.log &&
timeout -k 10 200 python -u tools/uniform_bench.py
