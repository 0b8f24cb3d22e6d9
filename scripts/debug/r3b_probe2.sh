#!/bin/bash
# pair hand-off probe (two-CU split of br512lat), then the full GPU test suite
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 120 scripts/probes/pair_handoff > gpurun_out/r3_pair_handoff.log 2>&1 || { echo "probe rc=$?"; cat gpurun_out/r3_pair_handoff.log; exit 1; }
cat gpurun_out/r3_pair_handoff.log
timeout -k 10 200 python scripts/debug/time_pbs_small.py 2>&1 | tail -1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3_gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r3_gpu_tests.log
exit $rc
