#!/bin/bash
# pair hand-off probe, then the 1-GPU bench line + rocprofv3 stats + PMC passes (scripts/bench_profile.sh)
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 120 scripts/probes/pair_handoff > gpurun_out/r3_pair_handoff.log 2>&1 || { echo "probe rc=$?"; cat gpurun_out/r3_pair_handoff.log; exit 1; }
cat gpurun_out/r3_pair_handoff.log
STEPS=${STEPS:-5} bash scripts/bench_profile.sh
