set -o pipefail
cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_model8.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pbs8_kernel_variants or aes8_one_round" > gpurun_out/b1kw_tests2.log 2>&1 &&
PASSES=2 VARIANTS="nospill:: spill:spill.so:" TAE_B=8192 bash scripts/ab/ab.sh pbs8 > gpurun_out/ab_b1kw_spill.txt 2>&1
