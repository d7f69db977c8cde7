#!/bin/bash
# Round-5 A/B of two library builds on one box, interleaved (through gpurun): headline value and the P = 1
# partitioned rehearsal of each run into <tag>/summary.txt.   usage: bash tools/r05_ab_lib.sh <tag> <libA> <libB> [rounds]
set -e -o pipefail
O=gpurun_out/$1; A=$2; B=$3; mkdir -p "$O"
for i in $(seq 1 "${4:-2}"); do
  for L in "$A" "$B"; do
    n=$(basename "$(dirname "$L")")
    BFSX_LIB=$PWD/$L timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline \
      > "$O/${n}_$i.json" 2> "$O/${n}_$i.err"
    python3 -c "import json; d=json.load(open('$O/${n}_$i.json')); p=d.get('partitioned_p1') or {}; print('$n run $i:', round(d['value'],1), 'GTEPS t_bfs', round(d['t_bfs_ms_mean'],4), 'p1', round(p.get('value',0),1))" | tee -a "$O/summary.txt"
  done
done
