set -o pipefail
cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_gpu_model8.py -m gpu -x -v --timeout 120 --timeout-method thread -k "ggsw_fourier8 or bootstrap_from_bits8 or aes8_one_round or other_n1024" > gpurun_out/fft1k_tests.log 2>&1 &&
TAE_LIB_PATH=$PWD/tfhe-aes-2_amd/dbg/pf4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "pfks or circuit_bootstrap" > gpurun_out/pf4_tests.log 2>&1 &&
PASSES=3 VARIANTS="def:: pf0:pf0.so: pf4:pf4.so: pf12:pf12.so:" bash scripts/ab/ab.sh pfks1 > gpurun_out/ab_pfks_pf.txt 2>&1
