set -o pipefail
cd /root/repo
PASSES=2 CLOCK=1 bash scripts/ab/ab.sh pbs1 pbs1lat 2>&1 | tee gpurun_out/ab_lf.txt
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_batch.py > gpurun_out/lf_tests.log 2>&1; rc=$?
tail -30 gpurun_out/lf_tests.log
exit $rc
