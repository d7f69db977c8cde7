#!/bin/bash
# Kernel trace of the partitioned loop at P = 1 (RCCL communicator of one): rocprofv3 --kernel-trace --stats over
# a short `bench.py --dist` run; the kernel trace csv is kept for a per-level dispatch count.
#   usage: bash tools/r04_prof_dist.sh <tag>
set -e -o pipefail
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 RANK=0 LOCAL_RANK=0 WORLD_SIZE=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --dist --steps 1 --warmup 1 --roots 8 --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/prof" -name "*kernel_trace.csv" -exec cp {} "$OUT/kernel_trace.csv" \;
rm -rf "$OUT/prof"
echo done > "$OUT/DONE"
