#!/bin/bash
# Build debug variants of the product library (timing only: variants compute garbage on purpose)
# into tfhe-aes-2_amd/dbg/<name>.so; each name maps to -D flags for csrc/kernels.hip.
# usage: build_variants.sh name1=-DFLAG1 name2="-DFLAG2 -DFLAG3" ...
set -e
cd "$(dirname "$0")/../../tfhe-aes-2_amd"
make -s
mkdir -p dbg
X4FLAGS=$(make -s --no-print-directory -f Makefile -f - <<<'print-x4: ; @echo $(X4FLAGS)' print-x4)
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -w --offload-arch=gfx950 -munsafe-fp-atomics $flags -c csrc/kernels.hip -o dbg/$name.o &
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -w --offload-arch=gfx950 -munsafe-fp-atomics $X4FLAGS $flags -c csrc/br512x4_inst.hip -o dbg/$name.x4.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o dbg/$name.so dbg/$name.o dbg/$name.x4.o build/client.o build/model.o build/capi.o build/keyio.o -lpthread
  rm dbg/$name.o dbg/$name.x4.o
done
ls dbg
