#!/bin/bash
# time every library in tfhe-aes-2_amd/dbg on the small-batch PBS (one AES block = 128 bits), twice, alternating
cd /root/repo
for pass in 1 2; do
  for lib in tfhe-aes-2_amd/dbg/*.so; do
    TAE_LIB_PATH=$PWD/$lib timeout -k 10 200 python scripts/debug/time_pbs_small.py 2>&1 | tail -1 || exit 1
  done
done
