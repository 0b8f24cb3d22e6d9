#!/bin/bash
# 8-bit model: parity of the opt-in two-workgroups-per-CU br1024 variant (TAE_B1K_O2=1) and same-box
# PBS timing against the default at the CBS batch shape (8192) and the extract_bits shape (1024)
cd /root/repo
mkdir -p gpurun_out
TAE_B1K_O2=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_model8.py -x -q --timeout 240 --timeout-method thread -k "variants" > gpurun_out/o2_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/o2_tests.log; exit 1; }
tail -1 gpurun_out/o2_tests.log
for pass in 1 2; do
  for B in 8192 1024; do
    TAE_PBS_B=$B timeout -k 10 200 python scripts/debug/time_pbs8.py 2>&1 | tail -1 || exit 1
    TAE_B1K_O2=1 TAE_PBS_B=$B timeout -k 10 200 python scripts/debug/time_pbs8.py 2>&1 | sed 's/^/O2 /' | tail -1 || exit 1
  done
done
