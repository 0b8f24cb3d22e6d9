#!/bin/bash
# 8-bit model: parity of the in-tree library (tests/test_gpu_model8.py), then same-box PBS timing of
# tfhe-aes-2_amd/dbg/*.so at the CBS batch shape (8192) and the extract_bits shape (1024), three passes
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_model8.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ab8_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ab8_tests.log; exit 1; }
tail -1 gpurun_out/ab8_tests.log
for pass in 1 2 3; do
  for B in 8192 1024 256; do
    for lib in tfhe-aes-2_amd/dbg/*.so; do
      TAE_PBS_B=$B TAE_LIB_PATH=$PWD/$lib timeout -k 10 200 python scripts/debug/time_pbs8.py 2>&1 | tail -1 || exit 1
    done
  done
done
