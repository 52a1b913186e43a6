#!/bin/bash
# Build an A/B variant of librx.so in-tree (here, on the CPU) with extra defines, for tools/gpu_ab.sh with
# B="RX_LIB=$PWD/<pkg>/librx_<name>.so". usage: bash tools/build_variant.sh <name> -DRX_SOMETHING ...
set -e
PKG=development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
NAME=$1; shift
OUT=/tmp/rxv_$NAME; mkdir -p $OUT
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wno-unused-function -Wno-unused-variable $*"
for f in $PKG/csrc/*.hip; do /opt/rocm/bin/hipcc $FLAGS -c $f -o $OUT/$(basename $f .hip).o & done; wait
# the species translation units (csrc/rx_species.h, the Makefile's NS_LIST / NS_SPLIT)
for f in rx_kernels rx_bc; do for n in 3 4 5 6 7 8 9; do
  /opt/rocm/bin/hipcc $FLAGS -DRX_NS=$n -c $PKG/csrc/$f.hip -o $OUT/${f}_ns$n.o & done; wait; done
for f in $PKG/csrc/*.cpp; do g++ -O2 -std=c++17 -fPIC -ffp-contract=off -c $f -o $OUT/$(basename $f .cpp).host.o; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OUT/*.o -o $PKG/librx_$NAME.so -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $PKG/librx_$NAME.so
