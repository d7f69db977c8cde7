#!/bin/bash
# A/B of two libbfsx builds on the distributed harness at P = 1 (torch.distributed.run, RCCL communicator of
# one), interleaved, through gpurun:   bash tools/ab_dist.sh <tag> <libA> <libB> [rounds]
set -e -o pipefail
O=gpurun_out/$1; A=$2; B=$3; mkdir -p "$O"
for i in $(seq 1 "${4:-2}"); do
  for L in $A $B; do
    n=$(basename "$L" .so)
    BFSX_LIB=$PWD/$L timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $((29600 + i)) bench.py --gpus 1 --dist --steps 4 --warmup 1 \
      --levels-json "$O/${n}_$i.levels.json" > "$O/${n}_$i.json" 2> "$O/${n}_$i.err"
    python3 -c "import json; d=json.load(open('$O/${n}_$i.json')); print('$n run $i:', round(d['value'],1), 'GTEPS', round(d['t_bfs_ms_mean'],4), 'ms')" | tee -a "$O/summary.txt"
  done
done
