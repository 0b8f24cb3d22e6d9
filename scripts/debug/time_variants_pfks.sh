#!/bin/bash
cd "$(dirname "$0")/../.."
timeout -k 10 200 python scripts/debug/time_pfks.py 2>&1 | tail -1 || exit 1
for lib in tfhe-aes-2_amd/dbg/*.so; do
  TAE_LIB_PATH=$PWD/$lib timeout -k 10 200 python scripts/debug/time_pfks.py 2>&1 | tail -1 || exit 1
done
