#!/bin/bash
# round 3, first GPU call: new tests, VALU probe, PBS stage timing of the current tree
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_gpu_batch.py "tests/test_gpu_model8.py::test_pfks8_bit_exact" > gpurun_out/r3_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/r3_tests.log; exit 1; }
tail -5 gpurun_out/r3_tests.log
timeout -k 10 120 scripts/probes/valu_rates > gpurun_out/r3_valu.log 2>&1 || { echo "probe rc=$?"; exit 1; }
cat gpurun_out/r3_valu.log
timeout -k 10 200 python scripts/debug/time_pbs.py 2>&1 | tail -2
timeout -k 10 200 python scripts/debug/time_pbs_small.py 2>&1 | tail -2
