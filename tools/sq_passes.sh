#!/bin/bash
# SQ (wave state / instruction mix) counter passes for the pull kernel, one pass per counter group.
#   usage (through gpurun): bash tools/sq_passes.sh <tag> [kernel-regex]
# Summarise afterwards on the CPU side: python tools/sq_summary.py gpurun_out/<tag>
set -e -o pipefail
TAG=${1:-sq}
KRE=${2:-k_bu}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-p1"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT"; do
  timeout -s KILL 300 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" --output-format csv \
      -d "$OUT/pass$i" -o run -- $B > "$OUT/pass$i.log" 2>&1
  i=$((i+1))
done
echo done > "$OUT/DONE"
