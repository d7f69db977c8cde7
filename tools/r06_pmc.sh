#!/bin/bash
# Round-6 profiling session (same steps as rounds 3-5): smoke, the FETCH_SIZE / WRITE_SIZE calibration microbenchmark (plain run for the
# known bytes, then one PMC pass per counter), the default bench, per-level records, rocprofv3 kernel stats and
# the HBM PMC passes of the BFS kernels.  Every GPU step under its own time limit; the first failure ends it.
#   usage (through gpurun): bash tools/r06_pmc.sh <tag> [steps]
# Summarise afterwards on the CPU side:
#   python tools/fetch_calib_summary.py gpurun_out/<tag>/calib profiles/<tag>_fetch_calibration.json
#   python tools/pmc_summary.py <tag>
set -e -o pipefail
TAG=${1:-r04}
STEPS=${2:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT/calib"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
(cd bfs-with-mapreduce_amd/csrc && cat bfs_core.h kernels_push.hip kernels_pull.hip kernels_persist.hip kernels_level.hip kernels_dist.hip | sha256sum) > "$OUT/src_sha"
B="python3 bench.py --steps $STEPS --warmup 1 --no-cpu-baseline --no-p1"
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 120 tools/fetch_calib > "$OUT/calib/calib.json" 2> "$OUT/calib/calib.err"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib/pmc_fetch" -o run -- \
    tools/fetch_calib > "$OUT/calib/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib/pmc_write" -o run -- \
    tools/fetch_calib > "$OUT/calib/pmc_write.log" 2>&1
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 $B --levels-json "$OUT/levels.json" > "$OUT/bench_levels.json" 2> "$OUT/bench_levels.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- $B \
    > "$OUT/trace.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_bu|k_finalize|k_td|k_unpack|k_resolve_log" --output-format csv \
    -d "$OUT/pmc_fetch" -o run -- $B > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_bu|k_finalize|k_td|k_unpack|k_resolve_log" --output-format csv \
    -d "$OUT/pmc_write" -o run -- $B > "$OUT/pmc_write.log" 2>&1
echo done > "$OUT/DONE"
