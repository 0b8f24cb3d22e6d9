set -o pipefail
cd /root/repo
timeout -k 10 900 python -u -m pytest tests/test_gpu_model8.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/lf1k_tests.log 2>&1 &&
PASSES=3 VARIANTS="base:base.so: lf1k::" TAE_B=8192 bash scripts/ab/ab.sh pbs8 > gpurun_out/ab_lf1k.txt 2>&1 &&
TAE_LIB_PATH=$PWD/tfhe-aes-2_amd/dbg/b1kprof.so TAE_REPS=1 timeout -k 10 200 python scripts/ab/time_stage.py pbs8 > gpurun_out/b1kprof_lf.txt 2>&1 &&
TAE_LIB_PATH=$PWD/tfhe-aes-2_amd/dbg/x4prof.so TAE_REPS=1 timeout -k 10 200 python scripts/ab/time_stage.py pbs1 > gpurun_out/x4prof_lf.txt 2>&1
