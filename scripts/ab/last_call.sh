set -o pipefail
cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_model8.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pbs8_kernel_variants or eight_blocks" > gpurun_out/b1kw_tests4.log 2>&1 &&
PASSES=3 VARIANTS="lds1:: allstash:allstash.so:" TAE_B=8192 CLOCK=1 bash scripts/ab/ab.sh pbs8 > gpurun_out/ab_b1kw_lds1.txt 2>&1
