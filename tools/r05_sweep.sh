#!/bin/bash
# Round 5: direction-rule options swept on one box, the default interleaved between them (through gpurun):
#   bash tools/r05_sweep.sh <tag> <steps> <spec>...   spec: name:key=value[,key=value]  or  base
set -e -o pipefail
O=gpurun_out/$1; STEPS=$2; shift 2; mkdir -p "$O"
for spec in "$@"; do
  name=${spec%%:*}; opts=()
  if [ "$spec" != "$name" ]; then IFS=',' read -ra kv <<< "${spec#*:}"; for x in "${kv[@]}"; do opts+=(--option "$x"); done; fi
  timeout -k 10 300 python3 bench.py --steps "$STEPS" --warmup 1 --no-cpu-baseline --no-p1 "${opts[@]}" \
    > "$O/$name.json" 2> "$O/$name.err"
  python3 -c "import json; d=json.load(open('$O/$name.json')); print('$spec', round(d['value'],1), 'GTEPS', round(d['t_bfs_ms_mean'],4), 'ms')" | tee -a "$O/summary.txt"
done
