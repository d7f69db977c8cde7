#!/bin/bash
# Per-level times of knockout builds (results wrong by construction) next to the product build, interleaved:
#   usage: bash tools/r04_knockout.sh <tag> <lib> [<lib> ...]    then tools/level_breakdown.py on the outputs
set -e -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p "$OUT"
for i in 1 2; do
  for L in "$@"; do
    n=$(basename "$L" .so)
    BFSX_LIB=$PWD/$L timeout -k 10 200 python3 tools/knockout_levels.py "$OUT/${n}_$i.json" 2 > "$OUT/${n}_$i.out" 2> "$OUT/${n}_$i.err"
  done
done
python3 tools/level_breakdown.py "$OUT"/*.json > "$OUT/breakdown.txt"
