#!/bin/bash
# VALU probe (mixed-issue classes), PBS parity tests of the tree's library, then same-box timing of the
# tfhe-aes-2_amd/dbg variants (twice, alternating)
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 120 scripts/probes/valu_rates > gpurun_out/r3_valu2.log 2>&1 || { echo "probe rc=$?"; exit 1; }
tail -8 gpurun_out/r3_valu2.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 240 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for pass in 1 2; do
  for lib in tfhe-aes-2_amd/dbg/*.so; do
    TAE_LIB_PATH=$PWD/$lib timeout -k 10 200 python scripts/debug/time_pbs.py 2>&1 | tail -1 || exit 1
  done
done
