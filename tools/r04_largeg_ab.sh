#!/bin/bash
# largeG stand-in per-level latency of several library builds on one box, interleaved (tools/largeg_sweep.py).
#   usage: bash tools/r04_largeg_ab.sh <tag> <rounds> <lib> [<lib> ...]
set -e -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for i in $(seq 1 "$R"); do
  for L in "$@"; do
    echo "$(basename "$L" .so) round $i: $(BFSX_LIB=$PWD/$L timeout -k 10 200 python3 tools/largeg_sweep.py persist_blocks=auto 2>>"$OUT/err.log")" | tee -a "$OUT/largeg.txt"
  done
done
