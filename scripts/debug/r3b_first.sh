#!/bin/bash
# round 3 (session 2) first GPU call: VALU probe + PBS stage timing of the current tree
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 120 scripts/probes/valu_rates > gpurun_out/r3_valu.log 2>&1 || { echo "probe rc=$?"; exit 1; }
cat gpurun_out/r3_valu.log
timeout -k 10 200 python scripts/debug/time_pbs.py 2>&1 | tail -2
timeout -k 10 200 python scripts/debug/time_pbs_small.py 2>&1 | tail -2
