#!/bin/bash
# GPU-box: same-box A/B of the 8-bit model's PBS at one ciphertext per CU (br1024lat, extract_bits
# shape) and at the CBS batch (br1024, 2048) for every library in tfhe-aes-2_amd/dbg/*.so, twice.
cd "$(dirname "$0")/../.."
for pass in 1 2; do
  for lib in tfhe-aes-2_amd/dbg/*.so; do
    TAE_PBS_B=${PBS_B:-256} TAE_LIB_PATH=$PWD/$lib timeout -k 10 200 python scripts/debug/time_pbs8.py 2>&1 | tail -1 || exit 1
  done
done
