#!/bin/bash
# Round-3 GPU check: regression tests, the whole GPU suite, a default bench.  Every GPU step under its own
# timeout; the first failure ends the script.   usage (through gpurun): bash tools/r03_check.sh <tag> [bench steps]
set -e -o pipefail
TAG=${1:-r03a}
STEPS=${2:-10}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
PYT="python3 -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_regress.py > "$OUT/regress.log" 2>&1
timeout -k 10 700 $PYT -m gpu tests > "$OUT/gputests.log" 2>&1
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 400 python3 bench.py --steps "$STEPS" --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
echo done > "$OUT/DONE"
