set -o pipefail
cd /root/repo
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/lfc_tests.log 2>&1 &&
PASSES=3 VARIANTS="base:base.so: chunk::" bash scripts/ab/ab.sh pbs1 pbs1lat > gpurun_out/ab_lf_chunk.txt 2>&1
