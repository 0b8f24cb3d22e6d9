#!/bin/bash
# clamped-digit K layout: parity (stage tests incl. every PFKS layout, the 128-block batch) then PFKS timing
# default (4 slots, clamped) vs TAE_PFKS_LAYOUT=k5 (5 slots), three alternating passes
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batch.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pfks2_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/pfks2_tests.log; exit 1; }
tail -1 gpurun_out/pfks2_tests.log
for pass in 1 2 3; do
  timeout -k 10 200 python scripts/debug/time_pfks.py 2>&1 | tail -1 || exit 1
  TAE_PFKS_LAYOUT=k5 timeout -k 10 200 python scripts/debug/time_pfks.py 2>&1 | tail -1 || exit 1
done
