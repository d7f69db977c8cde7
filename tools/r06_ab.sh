#!/bin/bash
# Round-6 interleaved A/B of library builds on one box (through gpurun):
#   bash tools/r06_ab.sh <tag> <rounds> <lib dir>... [-- extra bench args]
# Each run: bench.py (no CPU row, no P=1 rehearsal) with BFSX_LIB=<dir>/libbfsx.so; one summary line per run.
set -e -o pipefail
TAG=$1; R=$2; shift 2
LIBS=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do LIBS+=("$1"); shift; done
[ "$1" = "--" ] && shift
O=gpurun_out/$TAG; mkdir -p "$O"
for i in $(seq 1 "$R"); do
  for L in "${LIBS[@]}"; do
    n=$(basename "$L")
    BFSX_LIB=$PWD/$L/libbfsx.so timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-p1 "$@" \
      --levels-json "$O/${n}_$i.levels.json" > "$O/${n}_$i.json" 2> "$O/${n}_$i.err"
    python3 -c "import json; d=json.load(open('$O/${n}_$i.json')); print('$n run $i:', round(d['value'],1), 'GTEPS t_bfs', round(d['t_bfs_ms_mean'],4), 'unpack', d['t_unpack_ms'], 'resolve', d['t_resolve_ms'], 'vwo', round(d['value_with_output'],1))" | tee -a "$O/summary.txt"
  done
done
