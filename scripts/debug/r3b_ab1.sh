#!/bin/bash
# PBS parity tests for the tree's library, then same-box timing of tfhe-aes-2_amd/dbg variants (twice, alternating)
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for pass in 1 2; do
  for lib in tfhe-aes-2_amd/dbg/*.so; do
    case $lib in *prof*) continue;; esac
    TAE_LIB_PATH=$PWD/$lib timeout -k 10 200 python scripts/debug/time_pbs.py 2>&1 | tail -1 || exit 1
  done
done
if [ -f tfhe-aes-2_amd/dbg/prof.so ]; then
  TAE_LIB_PATH=$PWD/tfhe-aes-2_amd/dbg/prof.so timeout -k 10 200 python scripts/debug/time_pbs.py > gpurun_out/x4prof.log 2>&1 || exit 1
  grep x4prof gpurun_out/x4prof.log | tail -16
fi
