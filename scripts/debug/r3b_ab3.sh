#!/bin/bash
# same-box PBS stage timing of the tfhe-aes-2_amd/dbg variants (three alternating passes); optional parity
# tests of one variant library (PARITY_LIB) first
cd /root/repo
mkdir -p gpurun_out
if [ -n "$PARITY_LIB" ]; then
  TAE_LIB_PATH=$PWD/$PARITY_LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -1 gpurun_out/ab_tests.log
fi
for pass in 1 2 3; do
  for lib in tfhe-aes-2_amd/dbg/*.so; do
    TAE_LIB_PATH=$PWD/$lib timeout -k 10 200 python scripts/debug/time_pbs.py 2>&1 | tail -1 || exit 1
  done
done
