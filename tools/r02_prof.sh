#!/bin/bash
# One profiling session: smoke, the default bench, per-level stats, rocprof kernel stats and the HBM PMC
# passes for the BFS kernels (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950), plus an L2 pass.
#   usage (through gpurun): bash tools/r02_prof.sh <tag> [steps]
# Summarise afterwards on the CPU side: python tools/pmc_summary.py <tag>
set -e -o pipefail
TAG=${1:-r02}
STEPS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps $STEPS --warmup 1 --no-cpu-baseline --no-p1"
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 $B --levels-json "$OUT/levels.json" > "$OUT/bench_levels.json" 2> "$OUT/bench_levels.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B \
    > "$OUT/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_bu|k_finalize|k_td" --output-format csv \
    -d "$OUT/pmc_fetch" -o run -- $B > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_bu|k_finalize|k_td" --output-format csv \
    -d "$OUT/pmc_write" -o run -- $B > "$OUT/pmc_write.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "k_bu" --output-format csv \
    -d "$OUT/pmc_l2" -o run -- $B > "$OUT/pmc_l2.log" 2>&1
echo done > "$OUT/DONE"
