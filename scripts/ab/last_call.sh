set -o pipefail
cd /root/repo
PASSES=2 VARIANTS="def:: kreg3:kreg3.so: kreg2:kreg2.so: kreg0:kreg0.so:" TAE_B=8192 bash scripts/ab/ab.sh pbs8 > gpurun_out/ab_b1k_kreg.txt 2>&1
