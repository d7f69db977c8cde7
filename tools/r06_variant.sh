#!/bin/bash
# Build a variant of libbfsx.so with extra compile flags on kernels_level.hip (A/B of tuning constants):
#   bash tools/r06_variant.sh <out dir> "<-Dflags>"      (the other objects are the in-tree build's)
set -e
OUT=$1; FLAGS=$2; P=bfs-with-mapreduce_amd; B=$P/build
mkdir -p "$OUT/obj"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I include $FLAGS \
    -c $P/csrc/kernels_level.hip -o "$OUT/obj/kernels_level.o"
objs=$(for f in kernels_build kernels_push kernels_pull kernels_persist kernels_dist kernels_parse kernels_validate bfsx_api bfsx_comm; do echo $B/$f.o; done)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libbfsx.so" $objs "$OUT/obj/kernels_level.o" \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$OUT/obj"
