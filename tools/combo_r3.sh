set -o pipefail
bash tools/f32_ab.sh > /dev/null && tail -30 gpurun_out/f32_ab.log && bash tools/qr_ab_round3.sh | tail -30 && timeout -k 10 200 python -u -m pytest tests/test_gpu_concurrency.py -x -v --timeout 150 --timeout-method thread 2>&1 | tail -5
