#!/bin/bash
# Round-2 GPU check: the GPU suite (scale-30 partition tests separately, longer limit), then the default bench.
#   usage (through gpurun): bash tools/r02_check.sh <tag>
set -e -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    --deselect tests/test_gpu_scale30.py > "$OUT/gputests.log" 2>&1
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_scale30.py -x -v -s --timeout 240 --timeout-method thread \
    > "$OUT/scale30.log" 2>&1
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo done > "$OUT/DONE"
