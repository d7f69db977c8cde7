#!/bin/bash
# A/B timing of two builds of libbfsx on one box (through gpurun), each with optional bench options:
#   bash tools/ab_lib.sh <tag> <libA> <libB> [bench args...]
set -e -o pipefail
O=gpurun_out/$1; A=$2; B=$3; shift 3; mkdir -p $O
for i in 1 2 3; do
  for L in $A $B; do
    n=$(basename $L .so)
    BFSX_LIB=$PWD/$L timeout -k 10 200 python3 bench.py --steps 64 --warmup 4 --no-cpu-baseline "$@" \
      --levels-json $O/${n}_$i.levels.json > $O/${n}_$i.json 2> $O/${n}_$i.err
  done
done
