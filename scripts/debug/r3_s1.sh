#!/bin/bash
# GPU box: shortint_1bit model tests
cd /root/repo && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_gpu_shortint1.py > gpurun_out/r3_s1.log 2>&1; rc=$?
tail -40 gpurun_out/r3_s1.log; exit $rc
