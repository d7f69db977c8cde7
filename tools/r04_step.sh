#!/bin/bash
# Round-4 change check (through gpurun): the named GPU test files, then an interleaved A/B of two library
# builds on the default bench (ab_lib.sh), then one bench line with per-level records of the current build.
# The first failure ends it.
#   usage: bash tools/r04_step.sh <tag> "<test files>" [<libA> <libB> [rounds]]
set -e -o pipefail
TAG=$1; TESTS=$2; A=$3; B=$4; R=${5:-3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread $TESTS > "$OUT/tests.log" 2>&1
fi
if [ -n "$A" ]; then
  for i in $(seq 1 "$R"); do
    for L in $A $B; do
      n=$(basename "$L" .so)
      BFSX_LIB=$PWD/$L timeout -k 10 200 python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-p1 \
        --levels-json "$OUT/${n}_$i.levels.json" > "$OUT/${n}_$i.json" 2> "$OUT/${n}_$i.err"
    done
  done
fi
timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
echo done > "$OUT/DONE"
