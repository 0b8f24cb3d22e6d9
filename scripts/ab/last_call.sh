set -o pipefail
cd /root/repo
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 &&
bash scripts/bench_profile.sh > gpurun_out/bench_profile.log 2>&1
