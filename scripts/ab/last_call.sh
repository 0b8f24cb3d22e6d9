set -o pipefail
cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_model8.py -m gpu -x -v --timeout 300 --timeout-method thread -k "eight_blocks" > gpurun_out/b1kw_tests3.log 2>&1
