set -o pipefail
cd /root/repo
TAE_LIB_PATH=$PWD/tfhe-aes-2_amd/dbg/help.so timeout -k 10 300 python -u -m pytest tests/test_gpu_model8.py -m gpu -x -v --timeout 120 --timeout-method thread -k "pbs8_kernel_variants or aes8_one_round or bootstrap_from_bits8" > gpurun_out/help_tests.log 2>&1 &&
PASSES=3 VARIANTS="def:: help:help.so:" TAE_B=8192 bash scripts/ab/ab.sh pbs8 > gpurun_out/ab_b1k_help.txt 2>&1 &&
PASSES=2 VARIANTS="def:: help:help.so:" TAE_B=1024 bash scripts/ab/ab.sh pbs8 >> gpurun_out/ab_b1k_help.txt 2>&1
