set -o pipefail
cd /root/repo
TAE_LIB_PATH=$PWD/tfhe-aes-2_amd/dbg/rprof.so TAE_REPS=1 timeout -k 10 200 python scripts/ab/time_stage.py pbs8 > gpurun_out/b1krprof.txt 2>&1 &&
PASSES=2 VARIANTS="lvl::TAE_B1K_ROUNDS=0 rnd:: rndi2:rndi2.so:" TAE_B=8192 bash scripts/ab/ab.sh pbs8 > gpurun_out/ab_b1kr2.txt 2>&1
