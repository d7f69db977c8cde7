#!/bin/bash
# Round 6: HBM counters of the unpack kernels (k_unpack_live, k_unpack_gather, k_resolve_log), one PMC pass each.
#   usage (through gpurun): bash tools/r06_pmc_unpack.sh <tag>
set -e -o pipefail
TAG=${1:-r06pu}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-p1"
R="k_unpack|k_resolve_log|k_orig_nbrs"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --kernel-include-regex "$R" --output-format csv -d "$OUT/trace" -o run -- $B \
    > "$OUT/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$R" --output-format csv \
    -d "$OUT/pmc_fetch" -o run -- $B > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$R" --output-format csv \
    -d "$OUT/pmc_write" -o run -- $B > "$OUT/pmc_write.log" 2>&1
echo done > "$OUT/DONE"
