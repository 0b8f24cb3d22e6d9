#!/bin/bash
# same-box timing of the one-block PBS launch (128 ciphertexts, br512lat) for tfhe-aes-2_amd/dbg/*.so,
# three alternating passes
cd /root/repo
for pass in 1 2 3; do
  for lib in tfhe-aes-2_amd/dbg/*.so; do
    TAE_LIB_PATH=$PWD/$lib timeout -k 10 200 python scripts/debug/time_pbs_small.py 2>&1 | tail -1 || exit 1
  done
done
