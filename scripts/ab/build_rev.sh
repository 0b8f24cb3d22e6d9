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
objs=dbg/$name.o
if [ -f "$tmp/tfhe-aes-2_amd/csrc/br512x4_inst.hip" ]; then  # revisions with br512x4 in its own unit
  x4=$(git -C "$ROOT" show "$rev:tfhe-aes-2_amd/Makefile" | sed -n 's/^X4FLAGS = //p')
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -w --offload-arch=gfx950 -munsafe-fp-atomics $x4 "$@" \
    -c "$tmp/tfhe-aes-2_amd/csrc/br512x4_inst.hip" -o dbg/$name.x4.o
  objs="$objs dbg/$name.x4.o"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o dbg/$name.so $objs build/client.o build/model.o build/capi.o build/keyio.o -lpthread
rm -rf dbg/$name.o dbg/$name.x4.o "$tmp"
echo "dbg/$name.so from $rev"
