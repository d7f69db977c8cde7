#!/bin/bash
# Option sweep of the default bench (no CPU baseline, no P=1 rehearsal): one line per configuration.
#   usage: bash tools/r02_sweep.sh <tag> "<opts1>" "<opts2>" ...   (opts: space-separated key=value)
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for cfg in "$@"; do
  args=""
  for kv in $cfg; do args="$args --option $kv"; done
  timeout -k 10 200 python3 bench.py --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline --no-p1 $args \
      > "$OUT/cfg$i.json" 2> "$OUT/cfg$i.err"
  python3 -c "import json,sys;d=json.loads(open('$OUT/cfg$i.json').read().strip().splitlines()[-1]);print('$cfg'.ljust(40), round(d['value'],1), round(d['t_bfs_ms_mean'],4))" | tee -a "$OUT/summary.txt"
  i=$((i+1))
done
echo done > "$OUT/DONE"
