#!/bin/bash
# Round-3 change check (through gpurun): the named GPU test files, then an interleaved A/B of one option on
# the default bench, then per-level records with the option's B value.  The first failure ends it.
#   usage: bash tools/r03_step.sh <tag> "<test files>" <key> <valueA> <valueB> [rounds]
set -e -o pipefail
TAG=$1; TESTS=$2; KEY=$3; A=$4; B=$5; R=${6:-3}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread $TESTS > "$OUT/tests.log" 2>&1
fi
if [ -n "$KEY" ]; then
  bash tools/ab_option.sh "$TAG" "$KEY" "$A" "$B" "$R"
  timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-p1 --option "$KEY=$B" \
      --levels-json "$OUT/levels_$B.json" > "$OUT/levels_bench_$B.json" 2> "$OUT/levels_bench_$B.err"
  timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-p1 --option "$KEY=$A" \
      --levels-json "$OUT/levels_$A.json" > "$OUT/levels_bench_$A.json" 2> "$OUT/levels_bench_$A.err"
fi
echo done > "$OUT/DONE"
