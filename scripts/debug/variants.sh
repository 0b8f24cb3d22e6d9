#!/bin/bash
# run vp_steps.py against the default library and each debug variant under tfhe-aes-2_amd/dbg/
cd "$(dirname "$0")/../.."
for lib in tfhe-aes-2_amd/tfhe_aes/libtfhe_aes_amd.so tfhe-aes-2_amd/dbg/*.so; do
  echo "=== $lib"
  TAE_LIB_PATH=$PWD/$lib timeout -k 10 200 python scripts/debug/vp_steps.py 2>&1 | grep "^512 n_in 1 out 0\|^512 n_in 2 out 0" || exit 1
done
