#!/bin/bash
# Request-size-resolved fabric read counters (through gpurun): list the agent's counters, then -- if the
# 128-B request counter exists -- one pass of {TCC_EA0_RDREQ, TCC_EA0_RDREQ_32B, TCC_BUBBLE} over the
# calibration microbenchmark and over the bench's BFS kernels, so read bytes = 128*BUBBLE + 64*(RDREQ - BUBBLE
# - RDREQ_32B) + 32*RDREQ_32B need no per-access-class factor.   usage: bash tools/r03_pmc2.sh <tag>
set -e -o pipefail
TAG=${1:-r03p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
if grep -q "TCC_BUBBLE" "$OUT/avail.txt"; then
  C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum"
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$OUT/calib" -o run -- tools/fetch_calib \
      > "$OUT/calib.log" 2>&1
  timeout -s KILL 300 rocprofv3 --pmc $C --kernel-include-regex "k_bu|k_finalize|k_td" --output-format csv \
      -d "$OUT/bfs" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-p1 > "$OUT/bfs.log" 2>&1
fi
echo done > "$OUT/DONE"
