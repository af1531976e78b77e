# pending round-3 checks: single-precision / peer tests, then column-block tests + A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_single.py tests/test_gpu_peer.py -v --timeout 200 --timeout-method thread > gpurun_out/single_peer.log 2>&1
rc=$?
tail -4 gpurun_out/single_peer.log; grep FAILED gpurun_out/single_peer.log
[ $rc -le 1 ] || exit $rc
bash tools/cblk_ab.sh
