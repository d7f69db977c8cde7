#!/bin/bash
# Interleaved A/B of several library builds on the default bench (scale 26, 64 roots), one box.
#   usage: bash tools/r04_ab_multi.sh <tag> <rounds> <lib> [<lib> ...]      summary: python tools/ab_summary.py gpurun_out/<tag>
set -e -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in $(seq 1 "$R"); do
  for L in "$@"; do
    n=$(basename "$L" .so)
    BFSX_LIB=$PWD/$L timeout -k 10 200 python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-p1 \
      --levels-json "$OUT/${n}_$i.levels.json" > "$OUT/${n}_$i.json" 2> "$OUT/${n}_$i.err"
  done
done
