#!/bin/bash
# Build debug variants of the product library (timing only: variants compute garbage on purpose)
# into tfhe-aes-2_amd/dbg/<name>.so; each name maps to -D flags for csrc/kernels.hip.
# usage: build_variants.sh name1=-DFLAG1 name2="-DFLAG2 -DFLAG3" ...
set -e
cd "$(dirname "$0")/../../tfhe-aes-2_amd"
make -s
mkdir -p dbg
# the kernel units and their Makefile flag variables (kernels.hip: none); the variant flags go last
mkvar() { make -s --no-print-directory -f Makefile -f - <<<"print-var: ; @echo \$($1)" print-var; }
X4FLAGS=$(mkvar X4FLAGS); LATFLAGS=$(mkvar LATFLAGS); B1KFLAGS=$(mkvar B1KFLAGS); P16FLAGS=$(mkvar P16FLAGS)
HC="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -w --offload-arch=gfx950 -munsafe-fp-atomics"
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  $HC $flags -c csrc/kernels.hip -o dbg/$name.o &
  $HC $X4FLAGS $flags -c csrc/br512x4_inst.hip -o dbg/$name.x4.o &
  $HC $LATFLAGS $flags -c csrc/br512lat_inst.hip -o dbg/$name.lat.o &
  $HC $B1KFLAGS $flags -c csrc/br1024_inst.hip -o dbg/$name.b1k.o &
  $HC $P16FLAGS $flags -c csrc/br512p16_inst.hip -o dbg/$name.p16.o &
done
wait
for spec in "$@"; do
  name=${spec%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o dbg/$name.so dbg/$name.o dbg/$name.x4.o dbg/$name.lat.o dbg/$name.b1k.o dbg/$name.p16.o \
    build/client.o build/model.o build/capi.o build/keyio.o -lpthread
  rm dbg/$name.o dbg/$name.x4.o dbg/$name.lat.o dbg/$name.b1k.o dbg/$name.p16.o
done
ls dbg
