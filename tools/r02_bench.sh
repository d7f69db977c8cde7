#!/bin/bash
# scale-30 partition tests + the default bench (+ optional extra bench args)
set -e -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
if [ "${SKIP30:-0}" != 1 ]; then
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_scale30.py -x -v -s --timeout 240 --timeout-method thread \
    > "$OUT/scale30.log" 2>&1
fi
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
echo done > "$OUT/DONE"
