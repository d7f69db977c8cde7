#!/bin/bash
# A/B timing of one libbfsx option on the default bench (through gpurun), after a GPU test subset:
#   bash tools/opt_ab.sh <tag> <key> <valueA> <valueB> [pytest -k expression]
set -e -o pipefail
O=gpurun_out/$1; mkdir -p $O
if [ -n "$5" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$5" > $O/t.log 2>&1
fi
for i in 1 2 3; do
  for val in $3 $4; do
    timeout -k 10 200 python3 bench.py --steps 64 --warmup 4 --no-cpu-baseline --option $2=$val \
      --levels-json $O/${val}_$i.levels.json > $O/${val}_$i.json 2> $O/${val}_$i.err
  done
done
