#!/bin/bash
# Option sweep on the default bench (through gpurun): every "key=value[,key=value]" config, R interleaved rounds.
#   usage: bash tools/r04_sweep.sh <tag> <rounds> <config>...   (config "default" = no option)
set -e -o pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for i in $(seq 1 "$R"); do
  for C in "$@"; do
    OPTS=()
    if [ "$C" != "default" ]; then IFS=',' read -ra KV <<< "$C"; for kv in "${KV[@]}"; do OPTS+=(--option "$kv"); done; fi
    n=$(echo "$C" | tr '=,' '-_')
    timeout -k 10 200 python3 bench.py --steps 16 --warmup 2 --no-cpu-baseline --no-p1 "${OPTS[@]}" \
      --levels-json "$OUT/${n}_$i.levels.json" > "$OUT/${n}_$i.json" 2> "$OUT/${n}_$i.err"
  done
done
echo done > "$OUT/DONE"
