#!/bin/bash
# Interleaved sweep of one libbfsx option on the default bench (scale 26, 64 roots), one box.
#   usage: bash tools/r04_opt_sweep.sh <tag> <rounds> <key> <v1> [<v2> ...]     summary: python tools/ab_summary.py gpurun_out/<tag>
set -e -o pipefail
TAG=$1; R=$2; K=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in $(seq 1 "$R"); do
  for V in "$@"; do
    timeout -k 10 200 python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-p1 --option "$K=$V" \
      --levels-json "$OUT/${K}_${V}_$i.levels.json" > "$OUT/${K}_${V}_$i.json" 2> "$OUT/${K}_${V}_$i.err"
  done
done
