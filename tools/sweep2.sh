#!/bin/bash
# Sweep of option sets on the default bench (through gpurun), one line per run:
#   bash tools/sweep2.sh <tag> "<k=v k=v>" "<k=v>" ...   (each quoted argument is one option set)
set -e -o pipefail
O=gpurun_out/$1; shift; mkdir -p "$O"
i=0
for set in "$@"; do
  i=$((i + 1)); opts=""
  for kv in $set; do opts="$opts --option $kv"; done
  timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-p1 $opts \
    --levels-json "$O/run$i.levels.json" > "$O/run$i.json" 2> "$O/run$i.err"
  python3 -c "import json; d=json.load(open('$O/run$i.json')); print('[$set]', round(d['value'],1), 'GTEPS', round(d['t_bfs_ms_mean'],4), 'ms')" | tee -a "$O/summary.txt"
done
