#!/bin/bash
# GPU-box check: smoke() then the -m gpu parity/model suite (each step time-limited).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
rocm-smi --showproductname > gpurun_out/gpuinfo.txt 2>&1 || true
timeout -k 10 400 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "smoke failed: $?"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 ${GPU_TEST_TIMEOUT:-900} python -m pytest tests -q -m gpu ${PYTEST_ARGS:--x} > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log
exit $rc
