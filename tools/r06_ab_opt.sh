#!/bin/bash
# Round-6 interleaved A/B of option values on one box (through gpurun):
#   bash tools/r06_ab_opt.sh <tag> <rounds> "<opts A>" "<opts B>" ...   (each: space-separated key=value, or "-")
set -e -o pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
for i in $(seq 1 "$R"); do
  j=0
  for OPTS in "$@"; do
    j=$((j + 1)); args=()
    [ "$OPTS" != "-" ] && for kv in $OPTS; do args+=(--option "$kv"); done
    timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-p1 "${args[@]}" \
      --levels-json "$O/o${j}_$i.levels.json" > "$O/o${j}_$i.json" 2> "$O/o${j}_$i.err"
    python3 -c "import json; d=json.load(open('$O/o${j}_$i.json')); print('o$j [$OPTS] run $i:', round(d['value'],1), 'GTEPS t_bfs', round(d['t_bfs_ms_mean'],4), 'unpack', d['t_unpack_ms'], 'vwo', round(d['value_with_output'],1))" | tee -a "$O/summary.txt"
  done
done
