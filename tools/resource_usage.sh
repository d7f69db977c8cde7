#!/bin/bash
# Per-kernel VGPRs / scratch / occupancy of a HIP source (gfx950), one line per kernel.
#   usage: bash tools/resource_usage.sh bfs-with-mapreduce_amd/csrc/kernels_pull.hip [name-regex]
SRC=${1:?source}; PAT=${2:-.}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I "$(dirname "$0")/../include" -c "$SRC" -o /tmp/ru.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 |
    awk '/Function Name:/{n=$(NF-1)} / VGPRs:/{v=$(NF-1)} /ScratchSize/{s=$(NF-1)} /Occupancy/{print n, "vgpr=" v, "scratch=" s, "waves/simd=" $(NF-1)}' |
    grep -E "$PAT"
