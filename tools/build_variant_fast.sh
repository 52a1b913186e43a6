#!/bin/bash
# Like tools/build_variant.sh, but recompiles only the listed objects with the extra defines and links them with the
# main build's other objects (make first). usage: bash tools/build_variant_fast.sh <name> "<objects>" -DRX_X=1 ...
# objects: build/ names without .o, e.g. "rx_kernels rx_kernels_ns7" (species objects: <file>_ns<n>)
set -e
PKG=development-of-a-turbulent-numerical-solver-for-reactive-flows-in-su2_amd
NAME=$1; OBJS=$2; shift 2
OUT=/tmp/rxvf_$NAME; rm -rf $OUT; mkdir -p $OUT
cp $PKG/build/*.o $OUT/
FLAGS="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -Wno-unused-function -Wno-unused-variable $*"
for o in $OBJS; do
  src=${o%_ns*}; ns=""; [ "$src" != "$o" ] && ns="-DRX_NS=${o##*_ns}"
  /opt/rocm/bin/hipcc $FLAGS $ns -c $PKG/csrc/$src.hip -o $OUT/$o.o &
done; wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OUT/*.o -o $PKG/librx_$NAME.so -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $PKG/librx_$NAME.so
