#!/bin/bash
# Round-5 kernel trace of a short bench run (rocprofv3 --kernel-trace --stats), summary in gpurun_out/<tag>/
#   usage (through gpurun): bash tools/r05_prof.sh <tag> [bench args...]
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
(cd bfs-with-mapreduce_amd/csrc && cat bfs_core.h kernels_push.hip kernels_pull.hip kernels_persist.hip kernels_level.hip kernels_dist.hip | sha256sum) > "$OUT/src_sha"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-p1 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
find "$OUT/prof" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
echo done > "$OUT/DONE"
