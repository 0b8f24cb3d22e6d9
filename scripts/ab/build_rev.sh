#!/bin/bash
# Build the product library of a git revision's csrc/ (host objects of the working tree) into
# tfhe-aes-2_amd/dbg/<name>.so, for same-box A/B against the working tree (scripts/ab/ab.sh).
# usage: build_rev.sh name rev [extra hipcc flags]
set -e
name=$1; rev=$2; shift 2
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
tmp=$(mktemp -d)
git -C "$ROOT" archive "$rev" tfhe-aes-2_amd/csrc include | tar -x -C "$tmp"
cd "$ROOT/tfhe-aes-2_amd"
make -s
mkdir -p dbg
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -w --offload-arch=gfx950 -munsafe-fp-atomics "$@" \
  -c "$tmp/tfhe-aes-2_amd/csrc/kernels.hip" -o dbg/$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o dbg/$name.so dbg/$name.o build/client.o build/model.o build/capi.o build/keyio.o -lpthread
rm -rf dbg/$name.o "$tmp"
echo "dbg/$name.so from $rev"
