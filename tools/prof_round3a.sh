set -o pipefail
timeout -k 10 120 ./tools/gather_probe > gpurun_out/gather_probe.log 2>&1 || exit 1
bash tools/profile.sh gpurun_out/prof_band10m band10m 20 || exit 1
bash tools/profile.sh gpurun_out/prof_uniform10m uniform10m 10 || exit 1
echo ok
