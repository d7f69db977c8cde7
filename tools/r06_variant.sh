#!/bin/bash
# Build a variant of libbfsx.so with extra compile flags (A/B of tuning constants and code variants):
#   bash tools/r06_variant.sh <out dir> "<-Dflags>" [sources...]
# The listed sources (default: kernels_level) are recompiled with the flags; the other objects are the in-tree
# build's.
set -e
OUT=$1; FLAGS=$2; shift 2
SRCS=("$@"); [ ${#SRCS[@]} -eq 0 ] && SRCS=(kernels_level)
P=bfs-with-mapreduce_amd; B=$P/build
mkdir -p "$OUT/obj"
for s in "${SRCS[@]}"; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I include $FLAGS \
      -c $P/csrc/$s.hip -o "$OUT/obj/$s.o" &
done
wait
objs=""
for f in kernels_build kernels_push kernels_pull kernels_persist kernels_level kernels_dist kernels_parse kernels_validate bfsx_api bfsx_comm; do
  if [ -f "$OUT/obj/$f.o" ]; then objs="$objs $OUT/obj/$f.o"; else objs="$objs $B/$f.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libbfsx.so" $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$OUT/obj"
