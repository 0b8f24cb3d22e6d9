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
# revisions with kernels in units of their own: each built with its Makefile flag variable
for unit in br512x4_inst:X4FLAGS br512lat_inst:LATFLAGS br1024_inst:B1KFLAGS br512p16_inst:P16FLAGS; do
  src=${unit%%:*}; var=${unit#*:}
  [ -f "$tmp/tfhe-aes-2_amd/csrc/$src.hip" ] || continue
  fl=$(git -C "$ROOT" show "$rev:tfhe-aes-2_amd/Makefile" | sed -n "s/^$var = //p")
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -w --offload-arch=gfx950 -munsafe-fp-atomics $fl "$@" \
    -c "$tmp/tfhe-aes-2_amd/csrc/$src.hip" -o dbg/$name.$src.o
  objs="$objs dbg/$name.$src.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o dbg/$name.so $objs build/client.o build/model.o build/capi.o build/keyio.o -lpthread
rm -rf $objs "$tmp"
echo "dbg/$name.so from $rev"
