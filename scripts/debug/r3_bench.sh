#!/bin/bash
# GPU box: default bench line (driver shape) into gpurun_out/bench_default.json
cd /root/repo && mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
