#!/bin/bash
# PFKS tile-order A/B: the tree's library and every tfhe-aes-2_amd/dbg variant, two alternating passes
cd /root/repo
mkdir -p gpurun_out
for pass in 1 2; do
  bash scripts/debug/time_variants_pfks.sh || exit 1
done
