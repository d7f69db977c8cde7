#!/bin/bash
# Round-5 A/B of one option on the default bench, interleaved on one box, with per-level records (through gpurun):
#   bash tools/r05_ab.sh <tag> <key> <valueA> <valueB> [rounds] [steps]
set -e -o pipefail
O=gpurun_out/$1; mkdir -p "$O"
for i in $(seq 1 "${5:-2}"); do
  for val in "$3" "$4"; do
    timeout -k 10 300 python3 bench.py --steps "${6:-10}" --warmup 2 --no-cpu-baseline --no-p1 --option "$2=$val" \
      --levels-json "$O/${val}_$i.levels.json" > "$O/${val}_$i.json" 2> "$O/${val}_$i.err"
    python3 -c "import json; d=json.load(open('$O/${val}_$i.json')); print('$2=$val run $i:', round(d['value'],1), 'GTEPS', round(d['t_bfs_ms_mean'],4), 'ms', 'unpack', d['t_unpack_ms'], 'resolve', d.get('t_resolve_ms'))" | tee -a "$O/summary.txt"
  done
done
