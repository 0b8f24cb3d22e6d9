#!/bin/bash
# GPU box: PBS parity (br512x4 / br512lat / split batch / 128-block batch) then same-box A/B timing of dbg/*.so
cd /root/repo && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_batch.py > gpurun_out/r3_pbs_check.log 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/r3_pbs_check.log; exit 1; }
tail -3 gpurun_out/r3_pbs_check.log
scripts/debug/r3_ab.sh
