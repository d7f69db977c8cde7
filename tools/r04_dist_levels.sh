#!/bin/bash
# Per-level records of the single-device loop and the partitioned loop at P = 1 (RCCL, one rank), same graph and
# roots, then tools/level_breakdown.py on both.   usage: bash tools/r04_dist_levels.sh <tag>
set -e -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 200 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-p1 --levels-json "$OUT/single.json" \
  > "$OUT/single_bench.json" 2> "$OUT/single.err"
MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 timeout -k 10 300 python3 bench.py --dist \
  --steps 4 --warmup 1 --no-cpu-baseline --levels-json "$OUT/dist.json" > "$OUT/dist_bench.json" 2> "$OUT/dist.err"
python3 tools/level_breakdown.py "$OUT/single.json" "$OUT/dist.json" > "$OUT/breakdown.txt"
