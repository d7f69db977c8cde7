#!/bin/bash
# Round-5 A/B/C of three library builds on one box, interleaved (through gpurun), headline only.
#   usage: bash tools/r05_ab3_lib.sh <tag> <libA> <libB> <libC> [rounds]
set -e -o pipefail
O=gpurun_out/$1; mkdir -p "$O"
for i in $(seq 1 "${5:-2}"); do
  for L in "$2" "$3" "$4"; do
    n=$(basename "$(dirname "$L")")
    BFSX_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-p1 \
      > "$O/${n}_$i.json" 2> "$O/${n}_$i.err"
    python3 -c "import json; d=json.load(open('$O/${n}_$i.json')); print('$n run $i:', round(d['value'],1), 'GTEPS t_bfs', round(d['t_bfs_ms_mean'],4))" | tee -a "$O/summary.txt"
  done
done
