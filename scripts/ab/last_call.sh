set -o pipefail
cd /root/repo
bash scripts/gpu_check.sh > gpurun_out/check.txt 2>&1 &&
NB=64 bash scripts/prof8.sh > gpurun_out/prof8.txt 2>&1 &&
PROFILE=1 STEPS=2 bash scripts/bench_profile.sh > gpurun_out/bench_profile.txt 2>&1
