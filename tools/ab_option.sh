#!/bin/bash
# A/B of one libbfsx option on the default bench, interleaved, on one box (through gpurun):
#   bash tools/ab_option.sh <tag> <key> <valueA> <valueB> [rounds]
set -e -o pipefail
O=gpurun_out/$1; mkdir -p "$O"
for i in $(seq 1 "${5:-3}"); do
  for val in "$3" "$4"; do
    timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-p1 --option "$2=$val" \
      > "$O/${val}_$i.json" 2> "$O/${val}_$i.err"
    python3 -c "import json,sys; d=json.load(open('$O/${val}_$i.json')); print('$2=$val run $i:', round(d['value'],1), 'GTEPS', round(d['t_bfs_ms_mean'],4), 'ms')" | tee -a "$O/summary.txt"
  done
done
