#!/bin/bash
# GPU suite without the scale-30 tests, then the bench (optionally with extra args in $BENCH_ARGS)
set -e -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    --deselect tests/test_gpu_scale30.py > "$OUT/gputests.log" 2>&1
timeout -k 10 400 python3 bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
echo done > "$OUT/DONE"
